"""Failure path of the persistent GRU sweeps (gru_xcd.hip, gru_seq.hip) end to end.

SRNN_PERSIST_FORCE_FAIL=1 (a test switch read at each launch) makes one workgroup withhold
its hand-offs and shortens the spin limit, so the real give-up path runs: the waiting
workgroups raise the per-call error word AND the per-device sticky flag (persist.hip); the
fused clip+Adam sees the flag on the device and skips the update (weights and Adam moments
unchanged); the Trainer's per-iteration check raises; the check clears the flag and the next
step trains normally.  Both persistent paths (XCD-grouped and gru_seq, SRNN_GRU_XCD=0).
"""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

DEV = 'cuda'


def _setup(seed=3):
    import model as M
    import optim
    torch.manual_seed(seed)
    m = M.SampleRNN([16, 4], 1, 256, True, 256, True, False, 5, 3)
    m.compute_dtype = torch.bfloat16
    pred = M.Predictor(m).to(DEV)
    opt = optim.gradient_clipping(torch.optim.Adam(pred.parameters(), lr=1e-3))
    B, T, L = 16, 256, 64
    g = torch.Generator().manual_seed(seed)
    inp = torch.randint(0, 256, (B, L + T - 1), generator=g).to(DEV)
    tgt = torch.randint(0, 256, (B, T), generator=g).to(DEV)
    cond = torch.rand(B, T // L, 5, generator=g, dtype=torch.float64).to(DEV)
    spk = (torch.arange(B) % 3).reshape(B, 1).to(DEV)
    return pred, opt, (inp, tgt, cond, spk)


def _step(pred, opt, batch):
    import nn as snn
    inp, tgt, cond, spk = batch
    opt.zero_grad()

    def closure():
        loss = snn.sequence_nll_loss_bits(pred(inp, True, cond, spk), tgt)
        loss.backward()
        return loss
    return opt.step(closure)


def _state(pred, opt):
    ps = [p.detach().clone() for p in pred.parameters()]
    ms = [opt.state[p]['exp_avg'].clone() for p in pred.parameters() if p in opt.state]
    return ps, ms


@pytest.mark.parametrize('path', ['xcd', 'seq'])
def test_forced_handoff_failure_skips_update_and_raises(hip, monkeypatch, path):
    if path == 'seq':
        monkeypatch.setenv('SRNN_GRU_XCD', '0')
        if not hip.gru_seq_supported(torch.bfloat16, 16, 256):
            pytest.skip('gru_seq not supported on this device')
    elif not hip.gru_xcd_work_bytes(torch.bfloat16, 16, 256):
        pytest.skip('gru_xcd not supported on this device')
    pred, opt, batch = _setup()
    _step(pred, opt, batch)                       # a good step: flag clear
    hip.check_persistent_errors()
    before = _state(pred, opt)
    monkeypatch.setenv('SRNN_PERSIST_FORCE_FAIL', '1')
    _step(pred, opt, batch)
    torch.cuda.synchronize()
    after = _state(pred, opt)
    for a, b in zip(before[0] + before[1], after[0] + after[1]):
        assert torch.equal(a, b), 'a failed step must not move weights or Adam moments'
    with pytest.raises(RuntimeError, match='gave up a hand-off'):
        hip.check_persistent_errors()
    hip.check_persistent_errors()                 # taken: cleared
    monkeypatch.delenv('SRNN_PERSIST_FORCE_FAIL')
    loss = _step(pred, opt, batch)
    hip.check_persistent_errors()
    assert np.isfinite(float(loss.detach()))
    moved = _state(pred, opt)
    assert any(not torch.equal(a, b) for a, b in zip(after[0], moved[0]))


def test_trainer_raises_on_forced_failure(hip, monkeypatch):
    """The Trainer checks the flag once per iteration: a forced failure stops training with
    an exception instead of continuing on invalid states."""
    if not hip.gru_xcd_work_bytes(torch.bfloat16, 16, 256):
        pytest.skip('gru_xcd not supported on this device')
    import nn as snn
    from trainer import Trainer
    pred, opt, (inp, tgt, cond, spk) = _setup(5)
    data = [(inp.cpu(), torch.ones(1), tgt.cpu(), cond.cpu(), spk.cpu())]
    tr = Trainer(pred, snn.sequence_nll_loss_bits, opt, data, True, None)
    tr.run(1)                                      # healthy epoch
    monkeypatch.setenv('SRNN_PERSIST_FORCE_FAIL', '1')
    with pytest.raises(RuntimeError, match='gave up a hand-off'):
        tr.run(1)
