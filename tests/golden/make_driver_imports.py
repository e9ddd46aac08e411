"""Fixture generator: every ``gym_pybullet_drones.*`` import of the reference's driver scripts.

Parses ``simulator/CTDECattleHerder.py``, ``DTDECattleHerder.py``, ``DTDEModelPlayback.py`` and ``test.py``
with ``ast`` (nothing is imported or executed) and writes ``driver_imports.json``: per import its module, the
names taken from it and the source line.  ``tests/test_driver_imports_cpu.py`` resolves each one with
``rl-cattle-herding_amd/`` first on ``sys.path``.  Run in the build container:

    python tests/golden/make_driver_imports.py [/root/reference]
"""
import ast
import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
DRIVERS = ("CTDECattleHerder.py", "DTDECattleHerder.py", "DTDEModelPlayback.py", "test.py")


def driver_imports(ref_root):
    out = []
    for name in DRIVERS:
        path = os.path.join(ref_root, "gym_pybullet_drones", "simulator", name)
        tree = ast.parse(open(path).read(), filename=path)
        for node in ast.walk(tree):
            if isinstance(node, ast.ImportFrom) and node.module and node.module.startswith("gym_pybullet_drones"):
                out.append({"driver": name, "line": node.lineno, "module": node.module,
                            "names": [a.name for a in node.names]})
            elif isinstance(node, ast.Import):
                for a in node.names:
                    if a.name.startswith("gym_pybullet_drones"):
                        out.append({"driver": name, "line": node.lineno, "module": a.name, "names": []})
    out.sort(key=lambda r: (r["driver"], r["line"]))
    return out


if __name__ == "__main__":
    ref = sys.argv[1] if len(sys.argv) > 1 else "/root/reference"
    rows = driver_imports(ref)
    with open(os.path.join(HERE, "driver_imports.json"), "w") as f:
        json.dump({"source": "reference gym_pybullet_drones/simulator/*.py, ast import statements",
                   "imports": rows}, f, indent=1)
    print(len(rows), "imports")
