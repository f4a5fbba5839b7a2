"""Parity of the MEASURED path: bench.py's bf16 TBPTT step (configs[1]: 3-tier dim 1024,
FS = [16, 4], cond 43, 6 speakers, B = 128 rows x T = 1024 -- the persistent XCD GRU sweeps,
LDS-resident L1 gather, position-major dTab scatter, gemm3 epilogues, fused clip+Adam)
against the fp32 HIP path, which is pinned to the reference's own goldens
(test_gpu_parity.py).  Same weights (bench.make_model's seed), same synthetic chunks
(bench.synth_batches), two TBPTT chunks (reset, then carried hidden state).

Tolerances (bf16 operands with fp32 accumulation), set from the MI355X measurement
(round 2: losses 6.6e-5 relative apart at most; gradient relative L2 error 0.2-0.5 % in the
sample-level MLP, 1-7 % in the tiers, growing with the bf16 roundings carried through the
recurrences, cosine >= 0.9978): the loss of each chunk (the 2nd and 3rd after clipped Adam
steps, the 3rd on carried hidden states) within 3e-4 relative; every parameter gradient of
the first chunk within 10 % relative L2 error and cosine >= 0.995 of the fp32 gradient.
"""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = 'cuda'


def _run(dtype, batches):
    import bench
    import nn as snn
    import optim
    _, pred = bench.make_model(dtype)
    pred = pred.to(DEV)
    opt = optim.gradient_clipping(torch.optim.Adam(pred.parameters(), lr=1e-3))
    losses, grads = [], None
    for n, (inp, reset, tgt, cnd, spk) in enumerate(batches):
        opt.zero_grad()

        def closure():
            lp = pred(inp, reset, cnd, spk)
            loss = snn.sequence_nll_loss_bits(lp, tgt)
            loss.backward()
            return loss
        if n == 0:
            # gradients of the first chunk, before the clamp + Adam
            loss = closure()
            grads = {k: p.grad.detach().float().cpu().clone()
                     for k, p in pred.named_parameters() if p.grad is not None}
            opt.zero_grad()
            pred.reset_hidden_states()
        losses.append(float(opt.step(closure).detach()))
    torch.cuda.synchronize()
    import samplernn_hip as H
    H.check_persistent_errors()
    return losses, grads


@pytest.mark.parametrize('B', [128, 64, 512])
def test_bench_bf16_step_matches_fp32(hip, B):
    """B = 128: configs[1]; 512: configs[3]'s global batch on one GPU (the strong-scaling
    N = 1 point, 4 row tiles per sweep group); 64: its per-GPU share at 8 GPUs."""
    import bench
    import model as M
    T, L = 1024, 64
    batches = bench.gpu_batches(bench.synth_batches(B, T, L, 3, 0), DEV)
    l32, g32 = _run(torch.float32, batches)
    before = dict(M._STATS)
    l16, g16 = _run(torch.bfloat16, batches)
    # the bf16 step ran the persistent XCD sweeps, never the per-step recurrence kernels
    assert M._STATS['gru_xcd_fwd'] > before['gru_xcd_fwd']
    assert M._STATS['gru_xcd_bwd'] > before['gru_xcd_bwd']
    assert M._STATS['gru_cell_steps'] == before['gru_cell_steps']
    assert M._STATS['gru_cell_bwd_steps'] == before['gru_cell_bwd_steps']
    # ... and the hidden layer's bias gradient came from the da2 GEMM's epilogue
    assert M._STATS['csum_epi'] > before['csum_epi']
    print('losses fp32', l32, 'bf16', l16)
    np.testing.assert_allclose(l16, l32, rtol=3e-4, atol=0)
    assert g16.keys() == g32.keys()
    worst = []
    for k in g32:
        a, b = g16[k].double().reshape(-1), g32[k].double().reshape(-1)
        nb = b.norm().item()
        if nb == 0.0:
            assert a.norm().item() == 0.0, k
            continue
        rel = (a - b).norm().item() / nb
        cos = (a @ b).item() / (a.norm().item() * nb)
        worst.append((rel, cos, k))
    worst.sort(reverse=True)
    for rel, cos, k in worst:
        print('%-60s rel %.4f cos %.6f' % (k, rel, cos))
    for rel, cos, k in worst:
        # the MLP's dense layers see no recurrence: bf16 operand rounding only (measured
        # <= 0.6 %, MI355X round 3); everything upstream of the GRU sweeps or the dTab
        # scatter carries the recurrences' roundings (measured <= 6.8 %, cos >= 0.9977)
        dense = k.startswith(('model.sample_level_mlp.hidden', 'model.sample_level_mlp.output'))
        assert rel < (0.01 if dense else 0.085) and cos >= 0.997, (k, rel, cos)


def test_bf16_csum_epilogue_vs_column_pass(hip, monkeypatch):
    """configs[1] bf16 chunk: the hidden layer's bias gradient from the da2 GEMM's epilogue
    column sums (default) against a separate column-sum pass over da2 (SRNN_CSUM_EPI=0):
    every other gradient unchanged (bit-identical: the speaker-embedding gradient is an
    ordered row sum since round 5, srnn_index_add_rows), the bias gradient within fp32
    summation-order rounding (1e-4 of the largest entry)."""
    import bench
    import model as M
    B, T, L = 128, 1024, 64
    batches = bench.gpu_batches(bench.synth_batches(B, T, L, 1, 0), DEV)
    before = M._STATS['csum_epi']
    _, g_epi = _run(torch.bfloat16, batches)
    assert M._STATS['csum_epi'] > before
    monkeypatch.setenv('SRNN_CSUM_EPI', '0')
    mid = M._STATS['csum_epi']
    _, g_pass = _run(torch.bfloat16, batches)
    assert M._STATS['csum_epi'] == mid
    key = 'model.sample_level_mlp.hidden.bias'
    for k in g_pass:
        if k != key:
            assert torch.equal(g_epi[k], g_pass[k]), k
    a, b = g_epi[key].double(), g_pass[key].double()
    print('hidden bias grad: max |diff| %.3g, max |g| %.3g' % ((a - b).abs().max(), b.abs().max()))
    assert (a - b).abs().max() <= 1e-4 * b.abs().max()
