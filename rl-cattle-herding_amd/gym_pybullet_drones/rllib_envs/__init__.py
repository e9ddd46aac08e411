# Overlay: modules this package does not define (e.g. control/, simulator/, utils/flockUtils.py) resolve
# from a reference checkout later on sys.path; this package's own modules come first.
__path__ = __import__("pkgutil").extend_path(__path__, __name__)
from gym_pybullet_drones.rllib_envs.MARLCattleAviary import MARLCattleAviary  # noqa: F401
