"""Benchmark of the SampleRNN hot path on MI355X (BASELINE.json metric).

One JSON line (rank 0).  `value` = aggregate TBPTT training throughput (audio samples
per second = ranks x B x T / step time) for configs[1]: 3-tier SampleRNN, dim 1024,
frame_sizes [16, 4], 6-speaker + 43-d Ahocoder conditioning, T = 1024, B = 128 rows per
GPU, bf16 MFMA (fp32 master weights / recurrences), one step = forward + backward +
(all-reduce) + clipped Adam.  Weak scaling: every rank owns its own 128 stream rows.
The line also carries `tbptt_steps_per_s`, the generation throughput of configs[2]
(128 utterances x 3 s per GPU, replicas only; `gen` = bf16 through the persistent sample
loop, `gen_fp32` = the parity-grade fp32 path), the roofline of the dominant kernel
(its launches inside the timed steps, bracketed by HIP events on the launching stream)
and a bounded CPU baseline.

  python bench.py [--gpus N] [--steps K] [--warmup W] [--no-gen] [--no-cpu]
"""
import argparse
import json
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.abspath(__file__))
PKG = os.path.join(ROOT, 'jalil-saboorizadeh-multi-speaker-neural-vocoder_amd')
for p in (PKG, os.path.join(ROOT, 'tests', 'golden')):
    if p not in sys.path:
        sys.path.insert(0, p)

METRIC = ('audio samples/sec gen (3-tier dim1024) + TBPTT steps/sec @1/2/4/8 GPU')
MI355X_HBM_TBS = 8.0          # TB/s spec (MI355X_MICROARCH.md)
MI355X_BF16_TFLOPS = 2500.0   # dense bf16 MFMA spec
MI355X_FP32_TFLOPS = 157.3    # fp32 MFMA / vector spec


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def make_model(dtype, seed=77977, frame_sizes=(16, 4), cond_dim=43):
    import model as M
    torch.manual_seed(seed)
    m = M.SampleRNN(list(frame_sizes), 1, 1024, True, 256, True, False, cond_dim, 6)
    m.compute_dtype = dtype
    pred = M.Predictor(m)
    return m, pred


def synth_batches(B, T, L, n_chunks, row0, seed=0):
    """Stateful TBPTT layout (dataset.py:155-163, 242-289) on synthetic 16 kHz streams:
    sum of 3 sinusoids + Laplacian noise, float64 mu-law quantised, cond U[0,1), spk b%6."""
    import recipe
    import utils
    total = n_chunks * T + L
    audio = np.stack([recipe.synth_audio(total, seed + row0 + b) for b in range(B)])
    idx = utils.uquantize(torch.from_numpy(audio), 256)           # host, float64 path
    rng = np.random.Generator(np.random.PCG64(seed + 1000 + row0))
    cond = rng.uniform(0, 1, (B, n_chunks * T // L, 43))
    spk = ((np.arange(B) + row0) % 6).reshape(B, 1)
    out = []
    for n in range(n_chunks):
        inp = idx[:, n * T: n * T + L + T - 1].contiguous()
        tgt = idx[:, n * T + L: n * T + L + T].contiguous()
        cnd = torch.from_numpy(np.ascontiguousarray(cond[:, n * T // L:(n + 1) * T // L]))
        out.append((inp, n == 0, tgt, cnd, torch.from_numpy(spk)))
    return out


def gpu_batches(batches, dev):
    return [(a.to(dev), r, t.to(dev), c.to(dev), s.to(dev)) for a, r, t, c, s in batches]


def run_tbptt(args, dev, dist_mod):
    import nn as snn
    import optim
    B, T, L = args.batch, 1024, 64
    dtype = torch.bfloat16 if args.dtype == 'bf16' else torch.float32
    m, pred = make_model(dtype)
    pred = pred.to(dev)
    sync = dist_mod.GradAllReduce(overlap_groups=dist_mod.readiness_groups(pred)) \
        if dist_mod.world() > 1 else None
    opt = optim.gradient_clipping(torch.optim.Adam(pred.parameters(), lr=1e-3), grad_sync=sync)
    rows = slice(0, B)
    n_chunks = args.warmup + args.steps
    batches = gpu_batches(synth_batches(B, T, L, n_chunks, dist_mod.rank() * B), dev)
    losses = []

    def step(n):
        inp, reset, tgt, cnd, spk = batches[n]
        opt.zero_grad()     # fused clip+Adam: grads dropped, None == zero

        def closure():
            lp = pred(inp, reset, cnd, spk)
            loss = snn.sequence_nll_loss_bits(lp, tgt)
            loss.backward()
            return loss
        return opt.step(closure)

    for n in range(args.warmup):
        losses.append(step(n))
    torch.cuda.synchronize()
    dist_mod.barrier()
    torch.cuda.synchronize()
    import samplernn_hip as H
    # the roofline kernel's launches inside the timed steps, bracketed by HIP events on its
    # stream (two event records per step; model.py _MlpFn.forward)
    H.ROOF_EVENTS = []
    t0 = time.perf_counter()
    for n in range(args.warmup, n_chunks):
        losses.append(step(n))
    t_host = time.perf_counter() - t0      # enqueue time: close to dt when launch-bound
    torch.cuda.synchronize()
    dist_mod.barrier()
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    roof_ev, H.ROOF_EVENTS = H.ROOF_EVENTS, None
    kms_step = (sum(a.elapsed_time(b) for a, b in roof_ev) / len(roof_ev)) if roof_ev else None
    sys.stderr.write('tbptt host enqueue %.2f ms/step\n' % (t_host * 1e3 / max(args.steps, 1)))
    H.check_persistent_errors()            # (after the timed region) no hand-off given up
    if H.HOST_TIME:
        n_all = args.warmup + args.steps
        tot = sum(s for _, s in H.HOST_TIME.values())
        sys.stderr.write('host time in C entry points: %.2f ms/step (%d calls/step)\n' % (
            tot * 1e3 / n_all, sum(n for n, _ in H.HOST_TIME.values()) // n_all))
        for name, (n, s) in sorted(H.HOST_TIME.items(), key=lambda kv: -kv[1][1])[:30]:
            sys.stderr.write('  %-34s %6d calls %8.1f us/call\n' % (name, n, s * 1e6 / n))
    dt = dist_mod.max_over_ranks(dt, dev)
    loss_vals = [float(l.detach()) if torch.is_tensor(l) else float(l) for l in losses]
    return dt, loss_vals, pred, m, kms_step


def run_gen(args, dev, n_seqs, n_cond, dtype, frame_sizes=(16, 4), cond_dim=43):
    """One timed Generator call; returns (seconds, algorithmic weight elements read per
    generation step: the sample-level MLP every step, tier k once per nfs_k steps)."""
    import model as M
    m, _ = make_model(dtype, seed=4242, frame_sizes=frame_sizes, cond_dim=cond_dim)
    m = m.to(dev)
    w_step = sum(p.numel() for p in m.sample_level_mlp.parameters()) + sum(
        sum(p.numel() for p in t.parameters()) / t.n_frame_samples for t in m.frame_level_rnns)
    cond = torch.rand(n_seqs, n_cond, cond_dim, generator=torch.Generator().manual_seed(1))
    spk = np.arange(n_seqs) % 6
    gen = M.Generator(m, True)
    # warm-up (graph capture, kernel attributes) on a short run
    gen(n_seqs, 0, cond[:, :4], spk, sampler='philox', seed=5)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    gen(n_seqs, 0, cond, spk, sampler='philox', seed=5)
    torch.cuda.synchronize()
    return time.perf_counter() - t0, w_step


def kernel_roofline_gemm(dev, M, N, K, dtype, reps=20):
    """Average duration of the dominant GEMM launch (same shape/layout/dtype as in the
    step), timed with HIP events on the stream it is launched on."""
    import samplernn_hip as H
    a = torch.randn(M, K, device=dev).to(dtype)
    w = torch.randn(N, K, device=dev).to(dtype)
    bias = torch.zeros(N, device=dev)
    out = torch.empty(M, N, device=dev, dtype=dtype)
    for _ in range(10):
        H.linear(a, w, bias=bias, relu=True, out=out)
    s = torch.cuda.current_stream()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(s)
    for _ in range(reps):
        H.linear(a, w, bias=bias, relu=True, out=out)
    e1.record(s)
    e1.synchronize()
    ms = e0.elapsed_time(e1) / reps
    return ms


def pmc_traffic(kernel, path=os.path.join(ROOT, 'profiles', 'r02_pmc_gemm.txt')):
    """HBM bytes per launch of the roofline kernel from the committed rocprofv3 PMC passes
    (tools/roofline_kernel.py under --pmc FETCH_SIZE, then --pmc WRITE_SIZE): FETCH_SIZE kB x 2
    (gfx950 tallies 128-B requests at 64 B, MI355X_MICROARCH.md HBM section) + WRITE_SIZE kB."""
    try:
        vals = {}
        for line in open(path):
            m = line.split()
            if len(m) >= 6 and m[0] == 'avg':
                vals[m[1]] = float(m[-1])
        return int(round((2 * vals['FETCH_SIZE'] + vals['WRITE_SIZE']) * 1024))
    except (OSError, KeyError, ValueError):
        return None


def gru_sweep_roofline(dev, B=128, D=1024, Fr=64, reps=5):
    """MFMA utilisation of the recurrence's hidden x hidden products (the persistent XCD-grouped
    sweeps, gru_xcd.hip): the bottom tier's forward and backward sweep at the TBPTT step's shape
    (bf16, B rows, Fr frames), timed with HIP events on their stream; flop = Fr x 2 x B x 3D x D
    per sweep (the forward's W_hh h, the backward's W_hh^T dgh).  Latency-bound: one hand-off of
    h (dgh) between the group's workgroups per step."""
    import samplernn_hip as H
    T = torch.bfloat16
    g = torch.Generator(device=dev).manual_seed(3)
    whh = (torch.randn(3 * D, D, device=dev, generator=g) * 0.03).to(T)
    whh_t = whh.t().contiguous()
    bhh = torch.zeros(3 * D, device=dev)
    gi = torch.randn(B * Fr, 3 * D, device=dev, generator=g) * 0.5
    h0 = torch.zeros(B, D, device=dev)
    out = torch.empty(B, Fr, D, device=dev)
    outT = torch.empty(B, Fr, D, device=dev, dtype=T)
    gt = torch.empty(B, Fr, 4 * D, device=dev)
    nf = H.gru_xcd_work_bytes(T, B, D)
    nb = H.gru_xcd_bwd_work_bytes(T, B, D)
    if not nf or not nb:
        return None
    wf = torch.empty(nf, device=dev, dtype=torch.uint8)
    wb = torch.empty(nb, device=dev, dtype=torch.uint8)
    dy = torch.randn(B, Fr, D, device=dev, generator=g) * 0.1
    dgh = torch.empty(B, Fr, 3 * D, device=dev, dtype=T)
    dgi = torch.empty(B, Fr, 3 * D, device=dev, dtype=T)
    bsum = torch.empty(B, 4 * D, device=dev)
    ddir0 = torch.empty(B, D, device=dev)

    def fwd():
        H.lib().call('srnn_gru_xcd_fwd', H.BF16, B, D, Fr, H.ptr(gi), Fr * 3 * D, 3 * D,
                     H.ptr(h0), H.ptr(whh), H.ptr(bhh), H.ptr(out), H.ptr(outT), Fr * D, D,
                     H.ptr(gt), Fr * 4 * D, 4 * D, H.ptr(wf), nf, H.stream())

    def bwd():
        H.lib().call('srnn_gru_xcd_bwd2', H.BF16, B, D, Fr, H.ptr(dy), Fr * D, D, H.ptr(gt),
                     Fr * 4 * D, 4 * D, H.ptr(out), Fr * D, D, H.ptr(h0), H.ptr(whh_t), None,
                     H.ptr(dgh), None, H.ptr(dgi), H.ptr(bsum), Fr * 3 * D, 3 * D, H.ptr(ddir0),
                     H.ptr(wb), nb, H.stream())

    res = {}
    flop = Fr * 2.0 * B * 3 * D * D
    for name, fn in (('fwd', fwd), ('bwd', bwd)):
        for _ in range(2):
            fn()
        st = torch.cuda.current_stream()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(st)
        for _ in range(reps):
            fn()
        e1.record(st)
        e1.synchronize()
        ms = e0.elapsed_time(e1) / reps
        tf = flop / (ms * 1e-3) / 1e12
        res[name] = {'us_per_step': round(ms * 1e3 / Fr, 2), 'tflops': round(tf, 1),
                     'frac': round(tf / MI355X_BF16_TFLOPS, 4)}
    H.check_persistent_errors()
    return res


def gen_traffic(path=os.path.join(ROOT, 'profiles', 'r02_pmc_gen.txt')):
    """HBM bytes per generation step of the bf16 loop (B = 128, D = 1024, FS = [16, 4]) from the
    committed rocprofv3 PMC passes (tools/pmc_gen.py: FETCH_SIZE kB x 2 + WRITE_SIZE kB over
    every dispatch of the loop's kernels / samples generated)."""
    try:
        for line in open(path):
            m = line.split()
            if len(m) == 2 and m[0] == 'avg_step_bytes':
                return int(m[1])
    except (OSError, ValueError):
        pass
    return None


def cpu_baseline(seconds_budget=20.0):
    """The oracle (torch-CPU restatement of the reference) on the host cores: a bounded
    TBPTT sample of the same workload (config B dims, T = 1024, B = 4 rows)."""
    sys.path.insert(0, os.path.join(ROOT, 'oracle'))
    import samplernn_oracle as O
    threads = min(16, os.cpu_count() or 1)
    torch.set_num_threads(threads)
    m, pred = make_model(torch.float32)
    sd = {k: v.detach().clone() for k, v in pred.state_dict().items()}
    cfg = dict(frame_sizes=[16, 4], n_rnn=1, dim=1024, q_levels=256, weight_norm=False,
               cond_dim=43, spk_dim=6)
    om = O.from_state_dict(cfg, sd)
    names = [k for k, p in pred.named_parameters()]
    opt = O.OracleAdam([om.p[k] for k in names], lr=1e-3)
    B = 4
    batches = synth_batches(B, 1024, 64, 3, 0)
    O.tbptt_step(om, opt, names, batches[0])          # warm-up
    t0 = time.perf_counter()
    n = 0
    for b in batches[1:]:
        O.tbptt_step(om, opt, names, b)
        n += 1
        if time.perf_counter() - t0 > seconds_budget:
            break
    dt = time.perf_counter() - t0
    return {'value': round(n * B * 1024 / dt, 2), 'unit': 'samples/s', 'cores': threads,
            'kind': 'port',
            'sample': '%d TBPTT step(s) of the oracle (torch-CPU fp32 restatement) at config-B '
                      'dims, B=%d rows x T=1024, %d threads' % (n, B, threads)}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--gpus', type=int, default=1)
    ap.add_argument('--steps', type=int, default=10)
    ap.add_argument('--warmup', type=int, default=3)
    ap.add_argument('--batch', type=int, default=128)
    ap.add_argument('--dtype', default='bf16', choices=['bf16', 'fp32'])
    ap.add_argument('--gen-dtype', default='bf16', choices=['bf16', 'fp32'])
    ap.add_argument('--no-gen-fp32', action='store_true')
    ap.add_argument('--no-gen-e', action='store_true')
    ap.add_argument('--gen-seqs', type=int, default=128)
    ap.add_argument('--gen-cond', type=int, default=750)
    ap.add_argument('--no-gen', action='store_true')
    ap.add_argument('--no-cpu', action='store_true')
    args = ap.parse_args()

    import distributed as D
    D.init()
    dev = torch.device('cuda', D.device_index())
    torch.cuda.set_device(dev)
    N = D.world()
    if N != args.gpus:
        log('warning: --gpus %d but WORLD_SIZE %d' % (args.gpus, N))

    dt, losses, pred, m, kms_step = run_tbptt(args, dev, D)
    ms = dt / args.steps * 1000.0
    rows = args.batch
    samples = N * rows * 1024 * args.steps
    value = samples / dt
    log('tbptt: %.2f ms/step, losses %s' % (ms, ['%.3f' % l for l in losses]))
    del pred, m
    torch.cuda.empty_cache()

    # dominant kernel of the TBPTT step: the MLP hidden layer GEMM (B*T x D x D, bf16)
    tdt = torch.bfloat16 if args.dtype == 'bf16' else torch.float32
    M_, N_, K_ = rows * 1024, 1024, 1024
    # achieved: the hidden-layer GEMM's average launch inside the timed steps; the same shape
    # launched back to back in isolation (random operands, bias + ReLU) is reported beside it
    kms_iso = kernel_roofline_gemm(dev, M_, N_, K_, tdt)
    kms = kms_step if kms_step else kms_iso
    flops = 2.0 * M_ * N_ * K_
    ach = flops / (kms * 1e-3) / 1e12
    peak = MI355X_BF16_TFLOPS if args.dtype == 'bf16' else MI355X_FP32_TFLOPS
    roof = {'bound': 'mfma', 'achieved': round(ach, 1), 'peak': peak, 'unit': 'TFLOP/s',
            'frac': round(ach / peak, 4),
            'traffic': pmc_traffic('gemm3p_kernel') if (args.dtype == 'bf16' and rows == 128)
            else None,
            'traffic_algorithmic': 2 * (M_ * K_ + N_ * K_ + M_ * N_),
            'kernel': 'gemm3p_kernel (MLP hidden layer %dx%dx%d %s, bias + relu epilogue), '
                      '%.3f ms/launch inside the timed steps (%d launches, HIP events on its '
                      'stream); %.3f ms/launch isolated, back to back'
                      % (M_, N_, K_, args.dtype, kms, args.steps, kms_iso)}
    # MFMA utilisation of the GRU recurrence (north star: "MFMA utilisation for the GRU GEMMs")
    gru = None
    if args.dtype == 'bf16' and rows == 128:
        gru = gru_sweep_roofline(dev)
        if gru:
            gru.update({'bound': 'latency (one hand-off of h / dgh per step)', 'unit': 'TFLOP/s',
                        'peak': MI355X_BF16_TFLOPS,
                        'kernel': 'gru_xcd_fwd/bwd_kernel, bottom tier B=128 D=1024 64 frames'})

    def gen_line(dname, frame_sizes=(16, 4), cond_dim=43, n_cond=None, tag='3-tier dim1024 '
                 'FS=[16,4]'):
        gdt = torch.bfloat16 if dname == 'bf16' else torch.float32
        n_cond = n_cond or args.gen_cond
        L = int(np.prod(frame_sizes))
        t, W_step = run_gen(args, dev, args.gen_seqs, n_cond, gdt, frame_sizes, cond_dim)
        t = D.max_over_ranks(t, dev)
        gs = N * args.gen_seqs * n_cond * L / t
        steps_per_s = n_cond * L / t
        # algorithmic bytes per generation step: weights read once per step,
        # tiers amortised by their clocks (config C: 7,182,145 weights), + per-row activations
        es = 2 if dname == 'bf16' else 4
        bytes_step = es * W_step + args.gen_seqs * (4 * (1024 + 256) + 8 * 16 + 8)
        import samplernn_hip as H
        rows_pg = H.gen_persistent_rows(gdt, args.gen_seqs, 1024, 16)
        log('gen %s: %.3f s, %.0f samples/s (%.1fx realtime)' % (dname, t, gs, gs / 16000))
        return {'value': round(gs, 1), 'unit': 'samples/s', 'x_realtime': round(gs / 16000, 1),
                'x_realtime_per_gpu': round(gs / 16000 / N, 1), 'dtype': dname,
                'seconds': round(t, 3), 'steps_per_s': round(steps_per_s, 1),
                'us_per_step': round(1e6 / steps_per_s, 2),
                'sample_loop': ('persistent (gen_mlp.hip, %d rows/group)' % rows_pg) if rows_pg
                               else 'per-sample kernels (hipGraph)',
                'config': {'workload': 'generate %s cond %d, %d utt x %d cond rows (%d samples) '
                                       'per GPU, Philox sampler'
                                       % (tag, cond_dim, args.gen_seqs, n_cond, n_cond * L)},
                'roofline': {'bound': 'hbm',
                             'achieved': round(bytes_step * steps_per_s / 1e9, 1),
                             'peak': MI355X_HBM_TBS * 1000, 'unit': 'GB/s',
                             'frac': round(bytes_step * steps_per_s / 1e9 /
                                           (MI355X_HBM_TBS * 1000), 4),
                             'traffic': gen_traffic() if (dname == 'bf16' and tuple(frame_sizes)
                                                          == (16, 4) and args.gen_seqs == 128)
                                        else None}}

    gen = gen_fp32 = gen_e = None
    if not args.no_gen:
        gen = gen_line(args.gen_dtype)
        if args.gen_dtype != 'fp32' and not args.no_gen_fp32:
            gen_fp32 = gen_line('fp32')       # parity-grade numerics (bit-replay tests)
        if not args.no_gen_e:
            # configs[4]: 4-tier + look-ahead conditioning (C = 86), 1024 utterances over 8
            # GPUs = 128 per GPU (replicas), 188 cond rows x 256 = 48,128 samples each
            gen_e = gen_line(args.gen_dtype, (16, 4, 4), 86, 188,
                             '4-tier dim1024 FS=[16,4,4] look-ahead')

    cpu = None
    if D.rank() == 0 and N == 1 and not args.no_cpu:
        cpu = cpu_baseline()

    if D.rank() == 0:
        line = {'metric': METRIC, 'value': round(value, 1), 'unit': 'samples/s',
                'n_gpus': N, 'steps': args.steps, 'warmup': args.warmup,
                'ms_per_step': round(ms, 3), 'higher_is_better': True, 'scaling': 'weak',
                'vs_baseline': None, 'dtype': args.dtype, 'data': 'synthetic',
                'config': {'workload': 'TBPTT step, 3-tier SampleRNN dim1024 FS=[16,4] n_rnn=1 '
                                       'cond 43 spk 6, T=1024, B=%d rows/GPU, fwd+bwd+clip+Adam'
                                       % rows,
                           'global_batch': N * rows, 'seq_len': 1024,
                           'parallelism': 'dp%d' % N},
                'tbptt_steps_per_s': round(args.steps / dt, 3),
                'roofline': roof, 'cpu_baseline': cpu, 'gen': gen, 'gen_fp32': gen_fp32,
                'gen_config_e': gen_e, 'gru_sweep': gru,
                'final_loss': round(losses[-1], 4)}
        print(json.dumps(line), flush=True)
    D.barrier()


if __name__ == '__main__':
    main()
