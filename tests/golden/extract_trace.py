"""Extract the recorded PyBullet trace from the reference's ``evaluation_data.pkl`` WITHOUT unpickling.

Generator-side only (run in this container; the output ``trace_eval.npz`` is the committed fixture).

The file is written by ``evaluator.save_evaluation_data`` (reference
``gym_pybullet_drones/utils/evaluation.py:73-94``): a dict of lists of lists of numpy arrays.
Loading it with ``pickle`` would execute whatever the file names, so instead we walk its opcode
stream with ``pickletools.genops`` (a disassembler: it only decodes bytes) and interpret a small,
data-only subset ourselves: containers, scalars, byte strings, and the three numpy reconstruction
globals, which are turned into arrays by ``np.frombuffer`` on the raw bytes.  Any other global or
opcode aborts.  Nothing from the file is ever called or imported.
"""
import pickletools
import sys

import numpy as np

ALLOWED_GLOBALS = {("numpy.core.multiarray", "_reconstruct"), ("numpy", "ndarray"), ("numpy", "dtype"),
                   ("numpy.core.multiarray", "scalar"), ("collections", "OrderedDict")}


class _G:
    def __init__(self, mod, name):
        if (mod, name) not in ALLOWED_GLOBALS:
            raise ValueError(f"refusing global {mod}.{name}")
        self.key = (mod, name)


class _DT:
    def __init__(self, code):
        self.code = code
        self.order = "<"

    def np(self):
        return np.dtype(self.order + self.code if self.code[0] not in "<>|=" else self.code)


class _Arr:
    def __init__(self):
        self.value = None


def load_data_only(path):
    data = open(path, "rb").read()
    stack, memo, marks = [], {}, []

    def pop_mark():
        i = marks.pop()
        items = stack[i:]
        del stack[i:]
        return items

    for op, arg, _pos in pickletools.genops(data):
        n = op.name
        if n in ("PROTO", "FRAME"):
            continue
        elif n == "EMPTY_DICT":
            stack.append({})
        elif n == "EMPTY_LIST":
            stack.append([])
        elif n == "EMPTY_TUPLE":
            stack.append(())
        elif n == "MEMOIZE":
            memo[len(memo)] = stack[-1]
        elif n in ("BINGET", "LONG_BINGET"):
            stack.append(memo[arg])
        elif n == "MARK":
            marks.append(len(stack))
        elif n in ("SHORT_BINUNICODE", "BINUNICODE", "SHORT_BINBYTES", "BINBYTES", "BININT1", "BININT",
                   "BININT2", "BINFLOAT"):
            stack.append(arg)
        elif n == "NONE":
            stack.append(None)
        elif n == "NEWTRUE":
            stack.append(True)
        elif n == "NEWFALSE":
            stack.append(False)
        elif n == "STACK_GLOBAL":
            name = stack.pop()
            mod = stack.pop()
            stack.append(_G(mod, name))
        elif n == "TUPLE":
            stack.append(tuple(pop_mark()))
        elif n in ("TUPLE1", "TUPLE2", "TUPLE3"):
            k = int(n[-1])
            t = tuple(stack[-k:])
            del stack[-k:]
            stack.append(t)
        elif n == "REDUCE":
            args = stack.pop()
            fn = stack.pop()
            if not isinstance(fn, _G):
                raise ValueError("REDUCE on non-global")
            if fn.key == ("numpy.core.multiarray", "_reconstruct"):
                stack.append(_Arr())
            elif fn.key == ("numpy", "dtype"):
                stack.append(_DT(args[0]))
            elif fn.key == ("collections", "OrderedDict"):
                if args != ():
                    raise ValueError("OrderedDict with constructor arguments")
                stack.append({})   # filled by the SETITEMS that follow; key order is kept by dict
            elif fn.key == ("numpy.core.multiarray", "scalar"):
                dt, raw = args
                stack.append(np.frombuffer(raw, dtype=dt.np())[0])
            else:
                raise ValueError(f"unsupported reduce {fn.key}")
        elif n == "BUILD":
            state = stack.pop()
            obj = stack[-1]
            if isinstance(obj, _DT):
                obj.order = state[1] if state[1] in "<>" else "|"
            elif isinstance(obj, _Arr):
                _ver, shape, dt, _fortran, raw = state
                obj.value = np.frombuffer(raw, dtype=dt.np()).reshape(shape).copy()
            else:
                raise ValueError("BUILD on unsupported object")
        elif n == "APPENDS":
            items = pop_mark()
            stack[-1].extend(items)
        elif n == "APPEND":
            item = stack.pop()
            stack[-1].append(item)
        elif n == "SETITEMS":
            items = pop_mark()
            d = stack[-1]
            for i in range(0, len(items), 2):
                d[items[i]] = items[i + 1]
        elif n == "SETITEM":
            v = stack.pop()
            k = stack.pop()
            stack[-1][k] = v
        elif n == "STOP":
            break
        else:
            raise ValueError(f"unsupported opcode {n}")
    root = stack.pop()

    def fix(o):
        if isinstance(o, _Arr):
            return o.value
        if isinstance(o, list):
            return [fix(x) for x in o]
        if isinstance(o, tuple):
            return tuple(fix(x) for x in o)
        if isinstance(o, dict):
            return {k: fix(v) for k, v in o.items()}
        return o
    return fix(root)


def main(out="trace_eval.npz"):
    """Keep two whole episodes (time restarts at 0 at each reset): ep0 rows [0:453) and ep2 rows [1:602)."""
    d = load_data_only("/root/reference/gym_pybullet_drones/simulator/evaluation_data.pkl")
    segs = {"seg0": (0, 0, 453), "seg1": (2, 1, 602)}
    arrays = {}
    for name, (ep, a, b) in segs.items():
        t = np.array(d["time_per_step"][ep][a:b], dtype=np.float64)
        assert t[0] == 0.0 and np.all(np.diff(t) > 0), name
        arrays[name + "_drone_pos"] = np.stack(d["drone_poses_per_step"][ep][a:b]).astype(np.float64)
        arrays[name + "_cattle_pos"] = np.stack(d["cattle_poses_per_step"][ep][a:b]).astype(np.float64)
        arrays[name + "_drone_vel"] = np.stack(d["drone_vel_per_step"][ep][a:b]).astype(np.float64)
        arrays[name + "_cattle_vel"] = np.stack(d["cattle_vel_per_step"][ep][a:b]).astype(np.float64)
        arrays[name + "_time"] = t
        arrays[name + "_effectiveness"] = np.array(d["effectiveness_per_step"][ep][a:b], dtype=np.float64)
    np.savez_compressed(out, **arrays)
    for k, v in arrays.items():
        print(k, v.shape)


if __name__ == "__main__":
    main(*sys.argv[1:])
