"""CPU test of the batched RLlib multi-agent surface's host logic (cattleherd.marl_vec_env: agent keys, drop-out,
"__all__", the per-env agent bookkeeping) over the oracle-backed FakeBatch, against the reference's own MARL
rollouts (marl_roll_*.npz).  The GPU twin (tests/test_gpu_marl_vec.py) runs the same replay on the HIP batch."""
import pytest

from fake_batch import FakeBatch
from marl_replay import replay_marl_fixture


@pytest.fixture
def patched(monkeypatch):
    import cattleherd.marl_vec_env as mv
    monkeypatch.setattr(mv, "HerdBatch", FakeBatch)
    return mv


@pytest.mark.parametrize("fname", ["marl_roll_n3_m8_l0.npz", "marl_roll_n4_m16_l4.npz"])
def test_marl_vec_env_dicts_replay_reference_cpu(patched, fname):
    replay_marl_fixture(fname)
