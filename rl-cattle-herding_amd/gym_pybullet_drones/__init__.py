"""Drop-in replacement for the reference package's env surface (BenCooper305/RL-Cattle-Herding).

``gym_pybullet_drones.sb3_envs.CattleAviary`` and ``gym_pybullet_drones.rllib_envs.marl_wrapper.
RLlibMultiAgentWrapper`` keep the reference's constructors, attributes and reset/step contracts but
run on the MI355X HIP path (``cattleherd``).  Put ``rl-cattle-herding_amd/`` on PYTHONPATH ahead of
the reference and the drivers (simulator/CTDECattleHerder.py, DTDECattleHerder.py) run unchanged.
"""
