"""Co-residency of the persistent grids (csrc/handoff.hpp, persist.hip).

A persistent sweep (gru_xcd.hip) launches G x P workgroups that wait on each other's
hand-offs, so it is only correct once all of a group's members are resident.  The library
guarantees it: a launch is taken only when occupancy x CUs >= workgroups x processes sharing
the device (srnn_persist_check; otherwise refused with an error before anything runs), and
each member first waits for its whole group to arrive, bounded by wall time (30 s) rather
than by the hand-off spin count.  So a sweep that starts while other kernels hold CUs waits
for them and completes with the same bits -- it never spins out (the round-4 failure in
profiles/r04_dp2_rehearsal_303edb90.err.txt).  The CU holder is srnn_hold_cus (one
160-KiB-LDS workgroup per CU for a fixed wall time) on a second stream.
"""
import time

import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = 'cuda'


def _sweep_inputs(B, D, Fr, seed):
    T = torch.bfloat16
    g = torch.Generator().manual_seed(seed)
    whh = (torch.randn(3 * D, D, generator=g) * 0.03).to(DEV, T)
    bhh = (torch.randn(3 * D, generator=g) * 0.1).to(DEV)
    gi = (torch.randn(B, Fr, 3 * D, generator=g) * 0.5).to(DEV)
    h0 = (torch.randn(B, D, generator=g) * 0.5).to(DEV)
    return whh, bhh, gi, h0


def _sweep(hip, B, D, Fr, inp):
    whh, bhh, gi, h0 = inp
    T = torch.bfloat16
    nf = hip.gru_xcd_work_bytes(T, B, D)
    assert nf > 0
    wf = torch.empty(nf, device=DEV, dtype=torch.uint8)
    out = torch.empty((B, Fr, D), device=DEV)
    outT = torch.empty((B, Fr, D), device=DEV, dtype=T)
    gt = torch.empty((B, Fr, 4 * D), device=DEV)
    hp = torch.empty((B, Fr, D), device=DEV, dtype=T)
    hip.lib().call('srnn_gru_xcd_fwd2', hip.BF16, B, D, Fr, hip.ptr(gi), Fr * 3 * D, 3 * D,
                   hip.ptr(h0), hip.ptr(whh), hip.ptr(bhh), hip.ptr(out), hip.ptr(outT),
                   Fr * D, D, hip.ptr(gt), Fr * 4 * D, 4 * D, hip.ptr(hp), hip.ptr(wf), nf,
                   hip.stream())
    return wf, (out, outT, gt, hp)


@pytest.mark.parametrize('held', [128, 256])
def test_sweep_waits_for_cus_held_by_another_stream(hip, held):
    """A 256-workgroup sweep (B = 128, D = 1024: one workgroup per CU) enqueued while a kernel
    on another stream holds `held` CUs for 300 ms: the sweep waits (its late workgroups start
    when the holder ends), reports no failure and gives the bits of an unobstructed run."""
    B, D, Fr = 128, 1024, 64
    inp = _sweep_inputs(B, D, Fr, 5)
    wf, ref = _sweep(hip, B, D, Fr, inp)
    torch.cuda.synchronize()
    assert hip.lib().dll.srnn_gru_xcd_error(hip.ptr(wf)) == 0
    ref = [x.cpu() for x in ref]
    done = torch.zeros(1, device=DEV, dtype=torch.int32)
    side = torch.cuda.Stream()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    hip.lib().call('srnn_hold_cus', held, 300000, hip.ptr(done), side.cuda_stream)
    time.sleep(0.005)                      # the holder is on the CUs before the sweep starts
    wf2, got = _sweep(hip, B, D, Fr, inp)
    torch.cuda.synchronize()
    el = time.perf_counter() - t0
    assert int(done.item()) == held
    assert hip.lib().dll.srnn_gru_xcd_error(hip.ptr(wf2)) == 0
    hip.check_persistent_errors()          # sticky flag clear: no give-up anywhere
    print('sweep beside a %d-CU holder: %.0f ms end to end' % (held, el * 1e3))
    assert el >= 0.25                      # it did wait for the holder
    for a, b in zip(got, ref):
        assert torch.equal(a.cpu(), b)


def test_persistent_launch_refused_when_grid_cannot_fit(hip):
    """A persistent grid that cannot be resident for every process sharing the device is
    refused up front with an error (nothing launched): gru_seq at B = 128, D = 1024 is 256
    one-per-CU workgroups, which 8 processes sharing 256 CUs cannot all hold."""
    T = torch.bfloat16
    B, D, Fr = 128, 1024, 4
    try:
        hip.set_device_share(8)
        assert not hip.gru_seq_supported(T, B, D)
        assert hip.gru_xcd_work_bytes(T, B, D) > 0       # the XCD sweep re-lays itself out
        whh, bhh, gi, h0 = _sweep_inputs(B, D, Fr, 6)
        out = torch.empty((B, Fr, D), device=DEV)
        work = torch.zeros(1 << 16, device=DEV, dtype=torch.int32)
        with pytest.raises(RuntimeError, match='not supported|cannot all be resident'):
            hip.lib().call('srnn_gru_seq_fwd', hip.BF16, B, D, Fr, hip.ptr(gi), Fr * 3 * D,
                           3 * D, hip.ptr(h0), None, hip.ptr(whh), hip.ptr(bhh), hip.ptr(out),
                           None, Fr * D, D, None, 0, 0, hip.ptr(work), work.numel() * 4,
                           hip.stream())
        torch.cuda.synchronize()
    finally:
        hip.set_device_share(1)


@pytest.mark.parametrize('share', [2, 4])
def test_shared_device_sweeps_bit_identical(hip, share):
    """Declared sharing (distributed.init does it when ranks outnumber the GPUs) sizes every
    sweep launch to 1/share of the CUs -- B = 512 rows then run as chained launches of fewer
    groups -- with the same bits as the whole-device layout (rows are independent; the
    per-row arithmetic does not depend on the layout)."""
    B, D, Fr = 512, 1024, 9
    inp = _sweep_inputs(B, D, Fr, 7)
    _, ref = _sweep(hip, B, D, Fr, inp)
    ref = [x.cpu() for x in ref]
    try:
        hip.set_device_share(share)
        wf, got = _sweep(hip, B, D, Fr, inp)
        torch.cuda.synchronize()
        assert hip.lib().dll.srnn_gru_xcd_error(hip.ptr(wf)) == 0
    finally:
        hip.set_device_share(1)
    for a, b in zip(got, ref):
        assert torch.equal(a.cpu(), b)
