"""GPU tests of the runtime around the step kernel (through the C ABI): HIP-graph replay against
eager steps across reset/set_state/invalidate_obs, the device metric reduction against a host sum
of the per-env rows, and the sticky device error word of a failed LDS hand-off.

Reference anchors: the metrics are BaseAviary.update_evaluation_metrics' aggregate
(sb3_envs/BaseAviary.py:1406-1435); the error path stands in for an exception out of env.step
(marl_wrapper.py:87-95)."""
import ctypes

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _pair(mode, n, m, E, **kw):
    from cattleherd.env import HerdBatch
    return [HerdBatch(E, n, m, mode=mode, **kw) for _ in range(2)]


def _outs(h):
    return [x.clone() for x in (h.obs, h.reward, h.terminated, h.truncated, h.reset_happened)]


def _same(a, b):
    import torch
    return all(torch.equal(torch.nan_to_num(x.float(), nan=7.0), torch.nan_to_num(y.float(), nan=7.0))
               for x, y in zip(a, b))


@pytest.mark.parametrize("mode,n,m,E", [("ctde", 4, 16, 4096), ("marl", 3, 8, 300), ("ctde", 6, 16, 257)])
def test_graph_replay_equals_eager_across_state_changes(mode, n, m, E):
    """A graph captured once keeps matching eager steps after reset(), set_state() and
    invalidate_obs(): the Euler cache and the constant observation bytes are device words the
    kernel reads at run time (ch_internal.h StepParams::ctl), not values baked in at capture."""
    import torch
    K = 7
    eager, gr = _pair(mode, n, m, E, min_drones=2, max_drones=n)
    for h in (eager, gr):
        h.reset()
    graph = gr.capture_rollout(K, terminal_obs=False)
    for rnd in range(6):
        for _ in range(K):
            eager.step(random_actions=True, autoreset=True, terminal_obs=False)
        graph.replay()
        torch.cuda.synchronize()
        assert _same(_outs(eager), _outs(gr)), rnd
        s1, s2 = eager.get_state(), gr.get_state()
        for k in s1:
            assert np.array_equal(np.nan_to_num(s1[k]), np.nan_to_num(s2[k])), (rnd, k)
        if rnd == 1:
            for h in (eager, gr):
                h.reset()
        if rnd == 2:   # perturbed state injected into both (NUM_DRONES changes: dead rows move)
            s = eager.get_state()
            s["drone_quat"] = s["drone_quat"] + 1e-3
            s["drone_quat"] /= np.linalg.norm(s["drone_quat"], axis=-1, keepdims=True)
            s["n"] = np.where(np.arange(E) % 2 == 0, 2, n).astype(np.int32)
            s["active_mask"] = (1 << s["n"]) - 1
            for h in (eager, gr):
                h.set_state(s)
        if rnd == 3:
            for h in (eager, gr):
                h.obs.fill_(5.0)
                h.invalidate_obs()
    for h in (eager, gr):
        h.close()


def test_graph_replay_after_steps_into_another_obs_buffer():
    """Steps into a second observation buffer between replays of a graph captured on the first: envs that
    reset there (NUM_DRONES redrawn in [2, 6]) leave rows in the graph's buffer that the new episode no
    longer uses.  The buffer switch raises the per-env "constant bytes unknown" flags, so the next replay
    rewrites every block and the graph's buffer equals an eager twin stepped into one buffer only."""
    import torch
    E, n, m, K = 1024, 6, 16, 5
    eager, gr = _pair("ctde", n, m, E, min_drones=2, max_drones=n)
    for h in (eager, gr):
        h.reset()
    graph = gr.capture_rollout(K, terminal_obs=False)
    other = torch.full_like(gr.obs, 3.0)
    nres = 0
    for rnd in range(8):
        graph.replay()
        for _ in range(K):
            eager.step(random_actions=True, autoreset=True, terminal_obs=False)
        torch.cuda.synchronize()
        assert _same(_outs(eager), _outs(gr)), rnd
        for _ in range(30):   # eager twin: the same steps into its own buffer
            gr.step(random_actions=True, autoreset=True, terminal_obs=False, obs_out=other)
            eager.step(random_actions=True, autoreset=True, terminal_obs=False)
            nres += int(gr.reset_happened.sum())
        torch.cuda.synchronize()
        assert torch.equal(other, eager.obs), rnd
    assert nres > 50, nres
    for h in (eager, gr):
        h.close()


def test_full_reset_clears_the_device_error_word():
    """After a failed hand-off the handle reports CH_ERR_DEVICE until a full reset() rebuilds every env;
    then it steps and reports normally again (a masked reset does not clear it)."""
    import torch
    from cattleherd import _lib
    from cattleherd.env import HerdBatch
    b = HerdBatch(256, 4, 16, mode="ctde")
    b.reset()
    assert _lib.lib().ch__set_phase_mask(b.handle, ctypes.c_int32(64)) == 0
    b.step(random_actions=True)
    with pytest.raises(_lib.ChError):
        b.sync()
    assert _lib.lib().ch__set_phase_mask(b.handle, ctypes.c_int32(0)) == 0
    b.reset(mask=torch.ones(256, dtype=torch.uint8, device=b.device))
    with pytest.raises(_lib.ChError):
        b.sync()
    b.reset()
    b.sync()
    b.step(random_actions=True)
    b.sync()
    b.get_state()
    b.close()


def test_device_metrics_equal_host_sum_of_rows():
    """ch_metrics (device reduction + pinned copy) and ch_metrics_device agree with each other and
    with the metric rows summed on the host; reset_after zeroes the summed rows only."""
    import torch
    from cattleherd import _lib
    from cattleherd.env import HerdBatch
    E = 1000
    b = HerdBatch(E, 4, 16, mode="ctde", curriculum_level=2)
    b.reset()
    for _ in range(700):   # level 2 terminates on approach: episodes end inside the rollout
        b.step(random_actions=True, autoreset=True, terminal_obs=False)
    dev = b.metrics_device(reset=False)
    host = b.metrics(reset=False)
    torch.cuda.synchronize()
    assert np.array_equal(dev.cpu().numpy(), host)
    assert host[_lib.METRIC_NAMES.index("steps")] == E * 700 and host[1] > 0
    first = b.metrics(reset=True)
    assert np.array_equal(first, host)
    again = b.metrics(reset=False)
    assert np.all(again == 0)
    b.step(random_actions=True, autoreset=True, terminal_obs=False)
    assert b.metrics()[0] == E
    b.close()


def test_handoff_timeout_is_reported_not_silent():
    """A step whose LDS hand-off never completes (forced with the diagnostics phase bit 64) still
    ends -- every wait is bounded -- and the handle then reports CH_ERR_DEVICE from ch_sync and
    ch_metrics instead of returning wrong data silently.  A healthy handle reports nothing."""
    import torch
    from cattleherd import _lib
    from cattleherd.env import HerdBatch
    ok = HerdBatch(512, 4, 16, mode="ctde")
    bad = HerdBatch(512, 4, 16, mode="ctde")
    for h in (ok, bad):
        h.reset()
    assert _lib.lib().ch__set_phase_mask(bad.handle, ctypes.c_int32(64)) == 0
    for h in (ok, bad):
        h.step(random_actions=True)
    ok.sync()
    ok.metrics()
    with pytest.raises(_lib.ChError) as ei:
        bad.sync()
    assert ei.value.code == _lib.CH_ERR_DEVICE and "hand-off" in str(ei.value)
    with pytest.raises(_lib.ChError):
        bad.metrics()
    torch.cuda.synchronize()
    for h in (ok, bad):
        h.close()


def test_step_n_under_graph_capture():
    """ch_step_n inside a HIP graph capture records plain ch_step launches (no multi-step launch, no parameter
    upload in the graph): two replays equal 2 x K ch_step calls bit for bit, also after a ch_step_n of other io
    (which re-uploads the handle's parameter copy) ran between them."""
    import torch
    from cattleherd import _lib
    L = _lib.lib()
    a, b = _pair("ctde", 4, 16, 4096)
    for h in (a, b):
        h.reset()
        for _ in range(30):
            h.step(random_actions=True, autoreset=True, terminal_obs=False)
    torch.cuda.synchronize()
    K = 6
    m0 = L.ch__multi_steps(a.handle)
    side = torch.cuda.Stream(device=a.device)
    side.wait_stream(torch.cuda.current_stream(a.device))
    graph = torch.cuda.CUDAGraph()
    with torch.cuda.stream(side):
        with torch.cuda.graph(graph, stream=side):
            a.step_n(K, random_actions=True)
    torch.cuda.current_stream(a.device).wait_stream(side)
    torch.cuda.synchronize()
    assert L.ch__multi_steps(a.handle) == m0   # nothing ran, no multi-step launch recorded
    graph.replay()
    act = torch.zeros((4096, 4, 4), device=a.device)
    a.step_n(3, actions=act, random_actions=False)   # other parameters: the device copy is rewritten
    graph.replay()
    for _ in range(K):
        b.step(random_actions=True, autoreset=True, terminal_obs=False)
    b.step_n(3, actions=act, random_actions=False)
    for _ in range(K):
        b.step(random_actions=True, autoreset=True, terminal_obs=False)
    torch.cuda.synchronize()
    assert _same(_outs(a), _outs(b))
    sa, sb = a.get_state(), b.get_state()
    for k in sa:
        assert np.array_equal(np.asarray(sa[k]), np.asarray(sb[k]), equal_nan=True), k
    a.close()
    b.close()


@pytest.mark.parametrize("mode,n,m,E,autoreset", [("ctde", 4, 16, 4096, True), ("ctde", 4, 16, 4096, False),
                                                   ("marl", 4, 32, 4096, True), ("ctde", 2, 8, 1024, True)])
def test_step_n_given_actions(mode, n, m, E, autoreset):
    """ch_step_n with caller actions (the same action buffer every step, as n ch_step calls with it) and with
    auto-reset on or off: state, outputs and metrics equal to n ch_step calls bit for bit, the multi-step kernel ran."""
    import torch
    from cattleherd import _lib
    L = _lib.lib()
    a, b = _pair(mode, n, m, E)
    for h in (a, b):
        h.reset()
        for _ in range(60):
            h.step(random_actions=True, autoreset=True, terminal_obs=False)
    g = torch.Generator(device="cpu").manual_seed(5)
    act = (torch.rand((E, n, 4), generator=g) * 2 - 1).to(a.device)
    K = 17
    m0 = L.ch__multi_steps(a.handle)
    a.step_n(K, actions=act, autoreset=autoreset, random_actions=False)
    for _ in range(K):
        b.step(act, random_actions=False, autoreset=autoreset, terminal_obs=False)
    torch.cuda.synchronize()
    assert L.ch__multi_steps(a.handle) - m0 == K
    assert _same(_outs(a), _outs(b))
    sa, sb = a.get_state(), b.get_state()
    for k in sa:
        assert np.array_equal(np.asarray(sa[k]), np.asarray(sb[k]), equal_nan=True), k
    assert np.array_equal(a.metrics(), b.metrics(), equal_nan=True)
    a.close()
    b.close()


@pytest.mark.parametrize("mode,n,m,E,prec,multi,geom", [("ctde", 4, 16, 4096, "f64", True, None),
                                                        ("ctde", 2, 8, 4096, "f64", True, None),
                                                        ("ctde", 2, 8, 1024, "f64", True, None),
                                                        ("marl", 4, 32, 4096, "f64", True, None),
                                                        ("ctde", 4, 16, 4096, "f32", True, None),
                                                        ("ctde", 4, 16, 8200, "f32", True, None),
                                                        ("ctde", 3, 8, 300, "f64", False, None),
                                                        ("ctde", 4, 16, 4096, "f64", True, (8, 256)),
                                                        ("ctde", 4, 16, 1001, "f64", True, (8, 256))])
def test_step_n_equals_n_steps(mode, n, m, E, prec, multi, geom):
    """ch_step_n (k_step2_multi: each workgroup steps its envs back to back inside one launch) against the same number
    of ch_step calls: state, last outputs, metrics and the device-drawn actions bit for bit, with auto-resets inside the
    window (envs burnt in first so that episodes end at their long-run rate).  `multi`: the geometry has the multi-step
    kernel (the BASELINE ones); elsewhere ch_step_n falls back to one launch per step, with the same result.  `geom`:
    the multi-step handle runs that workgroup geometry (8-env workgroups, two per CU), the plain one the default.  f32
    at 8200 envs: more workgroups than CUs, the instantiation allocated for two workgroups per CU."""
    import ctypes
    import torch
    from cattleherd import _lib
    L = _lib.lib()
    a, b = _pair(mode, n, m, E, precision=prec)
    if geom is not None:
        assert L.ch__set_geometry(a.handle, ctypes.c_int32(geom[0]), ctypes.c_int32(geom[1])) == 0
    for h in (a, b):
        h.reset()
        for _ in range(140):
            h.step(random_actions=True, autoreset=True, terminal_obs=False)
    torch.cuda.synchronize()
    assert _same(_outs(a), _outs(b))
    K = 23
    m0 = L.ch__multi_steps(a.handle)
    ep0 = a.metrics()[1]
    a.step_n(K, random_actions=True)
    for _ in range(K):
        b.step(random_actions=True, autoreset=True, terminal_obs=False)
    torch.cuda.synchronize()
    assert (L.ch__multi_steps(a.handle) - m0 == K) == multi   # (the buffer's constant bytes are in place: no plain step)
    assert _same(_outs(a), _outs(b))
    assert torch.equal(a.actions, b.actions)
    sa, sb = a.get_state(), b.get_state()
    for k in sa:
        assert np.array_equal(np.asarray(sa[k]), np.asarray(sb[k]), equal_nan=True), k
    assert np.array_equal(a.metrics(), b.metrics(), equal_nan=True)
    # episodes ended (auto-resets) inside the window: CTDE at these sizes resets a few envs per step
    assert a.metrics()[1] > ep0 or mode == "marl"
    # a buffer whose constant observation bytes are unknown (invalidate_obs): one plain step first, then the kernel
    m1 = L.ch__multi_steps(a.handle)
    a.invalidate_obs()
    b.invalidate_obs()
    a.step_n(5, random_actions=True)
    for _ in range(5):
        b.step(random_actions=True, autoreset=True, terminal_obs=False)
    torch.cuda.synchronize()
    assert (L.ch__multi_steps(a.handle) - m1 == 4) == multi
    assert _same(_outs(a), _outs(b))
    sa, sb = a.get_state(), b.get_state()
    for k in sa:
        assert np.array_equal(np.asarray(sa[k]), np.asarray(sb[k]), equal_nan=True), k
    a.close()
    b.close()
