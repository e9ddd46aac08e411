"""Drop-in replacement for the reference package's env surface (BenCooper305/RL-Cattle-Herding).

``gym_pybullet_drones.sb3_envs.CattleAviary`` and ``gym_pybullet_drones.rllib_envs.marl_wrapper.
RLlibMultiAgentWrapper`` keep the reference's constructors, attributes and reset/step contracts but
run on the MI355X HIP path (``cattleherd``).  Put ``rl-cattle-herding_amd/`` on PYTHONPATH ahead of
the reference and the drivers (simulator/CTDECattleHerder.py, DTDECattleHerder.py) run unchanged.
"""
# Overlay: modules this package does not define (e.g. control/, simulator/, utils/flockUtils.py) resolve
# from a reference checkout later on sys.path; this package's own modules come first.
__path__ = __import__("pkgutil").extend_path(__path__, __name__)
