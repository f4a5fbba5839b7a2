"""Benchmark of the SampleRNN hot path on MI355X (BASELINE.json metric).

One JSON line (rank 0).  `value` = aggregate TBPTT training throughput (audio samples per
second = global batch x T / step time) of the drop-in Trainer.train (trainer/__init__.py:62-117,
the product path: forward, NLL, backward, DP all-reduce, fused clip + Adam, lagged failure
check) on a 3-tier SampleRNN, dim 1024, frame_sizes [16, 4], 6 speakers + 43-d Ahocoder
conditioning, T = 1024, bf16 MFMA with fp32 master weights / recurrences.  On one GPU the
Trainer runs in graph mode: the warm-up chunks run the eager steps and capture the step, the
timed chunks replay it (`graph_replays`; `eager_ms_per_step` = the same step enqueued kernel
by kernel, measured right after).

Default workload = configs[3]: global batch 512 stream rows sharded over the N ranks
(512 / N rows per GPU, strong scaling; N = 1 is the whole 512-row batch on one GPU).  Beside
it the line carries
  * `config_b` (N = 1): configs[1], 128 rows on one GPU;
  * `handwritten_only` (N = 1, bf16): the headline step with every GEMM on the hand-written
    kernels (SRNN_BLASLT=0);
  * `weak_64`: 64 rows per GPU (weak scaling at configs[3]'s 8-GPU share);
  * `weak_512` (N > 1): 512 rows per GPU, global batch 512 N (weak scaling at the N = 1
    headline's per-GPU work: only the all-reduce is added);
  * `roofline`: the step's DOMINANT kernel (largest time per step among the probed launch
    sites: GRU sweeps, dTab scatter, MLP hidden GEMM, fused clip + Adam), measured with HIP
    events on the launching stream around each launch over eager steps of the same run (a
    replayed graph runs the same kernels); `kernels` lists every probed site;
    `step_mfma`: executed MFMA work of the whole step / step time / bf16 peak;
  * generation throughput of configs[2] (`gen` bf16 persistent loop, `gen_fp32` the reference
    precision) and configs[4] (`gen_config_e`, `gen_config_e_fp32`), rows sharded over ranks (each rank its
    contiguous 1/N share of the utterances, no collective in the loop);
  * `cpu_baseline`: the oracle (torch-CPU restatement) on the host cores, bounded samples of
    the TBPTT step at configs[1]'s batch and of generation at configs[2]'s.

  python bench.py [--gpus N] [--steps K] [--warmup W] [--batch ROWS_PER_GPU] [--no-gen]

--gpus N > 1 outside torchrun spawns the N ranks itself (spawn_ranks: N child processes with
the torchrun environment, the parent touching no GPU); under torchrun (WORLD_SIZE set) each
process is one rank.  `n_gpus` is the process group's size, `rccl_ranks` the ranks of an RCCL
group (0 under gloo).
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
GLOBAL_B = 512                # configs[3]
T_SEQ, D_MODEL, FS, COND, SPK, Q = 1024, 1024, (16, 4), 43, 6, 256


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


def step_mfma_flops(B, T=T_SEQ, D=D_MODEL, fs=FS, C=COND, S=SPK, Q=Q, n_rnn=1):
    """MFMA work one TBPTT step executes (model.py's GEMMs and persistent sweeps, the folded
    L1: the table build replaces the reference's 4.2 M-MAC/sample input conv).  flop = 2 MAC."""
    f = 0.0
    nfs = list(np.cumprod(fs))
    for k, (fsz, n) in enumerate(zip(fs, nfs)):
        M = B * T // n                                    # rows x frames of tier k
        fwd = 2.0 * M * n * D                             # input_expand
        if k == len(fs) - 1:
            fwd += 2.0 * M * C * D + 2.0 * B * S * D      # cond_expand, spk_expand
        fwd += n_rnn * (2.0 * M * D * 3 * D) * 2          # GRU input projection + recurrence
        fwd += 2.0 * M * D * fsz * D                      # upsampling
        bwd = 2 * (2.0 * M * D * fsz * D)                 # upsampling dW + dX
        bwd += n_rnn * (2.0 * M * 3 * D * D * 4 + 2.0 * B * 3 * D * D)   # sweep, dW_hh,
        bwd += 2.0 * M * D * n                            # dW_ih, dX; dh0 / input dW
        if k == len(fs) - 1:
            bwd += 2.0 * M * D * C + 2 * 2.0 * B * D * S
        f += fwd + bwd
    BT, F0 = B * T, fs[0]
    f += 2.0 * F0 * Q * Q * D                             # Tab = Wp . E (forward)
    f += 2.0 * BT * D * D + 2.0 * BT * D * Q              # hidden, output
    f += 2 * 2.0 * BT * D * Q + 2 * 2.0 * BT * D * D      # their dW + dX
    f += 2 * 2.0 * F0 * D * Q * Q                         # dE, dWp from dTab
    return f


def site_roofline(site, ms, work_per_step, dtype_peak):
    """Roofline entry of one probed launch site: achieved = algorithmic work / its time."""
    if site in ('dtab_scatter', 'adam_clip', 'mlp_l1_gather'):
        ach = work_per_step / (ms * 1e-3) / 1e9
        return {'bound': 'hbm', 'achieved': round(ach, 1), 'peak': MI355X_HBM_TBS * 1000,
                'unit': 'GB/s', 'frac': round(ach / (MI355X_HBM_TBS * 1000), 4)}
    ach = work_per_step / (ms * 1e-3) / 1e12
    return {'bound': 'mfma', 'achieved': round(ach, 1), 'peak': dtype_peak, 'unit': 'TFLOP/s',
            'frac': round(ach / dtype_peak, 4)}


SITE_NOTES = {
    'gru_xcd_bwd': 'gru_xcd_bwd_pk_kernel: the GRU reverse sweeps (every tier, one persistent '
                   'launch each; dgh_{t+1} W_hh products; bound by reading the hand-off of dgh '
                   '(16 rows x D {3 x bf16, tag} granules per workgroup and step) from L2)',
    'gru_xcd_fwd': 'gru_xcd_fwd_kernel: the GRU forward sweeps (W_hh h products; one hand-off '
                   'of h per step)',
    'dtab_scatter': 'dtab_prep_kernel + dtab_pk_kernel: backward of the folded embedding.conv '
                    '(dTab scatter, two columns per 64-bit LDS atomic; bound by LDS atomic '
                    'issue, priced against HBM)',
    'mlp_hidden_gemm': 'gemm3p_kernel: sample-level MLP hidden layer (B*T x D x D, bias + '
                       'ReLU epilogue)',
    'adam_clip': 'adam_clip_multi_kernel: fused clamp + Adam over every parameter',
    'mlp_l1_gather': 'mlp_l1_lds_kernel: sample-level MLP input layer, the folded embedding.conv '
                     'table gathered from LDS + upper, a1 = ReLU(.) and its mask bits '
                     '(HBM: upper read, a1 written)',
    'mlp_da1_gemm': 'gemm3p_kernel: sample-level MLP input-activation gradient da1 = (da2 '
                    'W_hid) * [a1 > 0] (B*T x D x D, ReLU-mask epilogue, max |da1| for the '
                    'dTab scale)',
    'mlp_da2_gemm': 'gemm3p_kernel: sample-level MLP hidden-activation gradient da2 = (dz '
                    'W_out) * [a2 > 0] (B*T x D x Q, ReLU-mask epilogue, the hidden bias '
                    'gradient as per-block column sums)',
    'mlp_dw_hid_gemm': 'gemm3_kernel: sample-level MLP hidden weight gradient da2^T a1 '
                       '(D x D x B*T, fp32 out)',
}


class _LossLog:
    """Trainer 'iteration' plugin keeping a copy of every step's loss (a replayed graph step
    hands out the same static loss buffer each time)."""

    def __init__(self):
        self.trigger_interval = [(1, 'iteration')]
        self.values = []

    def register(self, trainer):
        pass

    def iteration(self, it, inputs, target, output, loss):
        self.values.append(loss.detach().clone())


def run_tbptt(dev, dist_mod, rows, steps, warmup, dtype, probe=True):
    """Warm-up then `steps` timed chunks of the drop-in Trainer.train on `rows` stream rows
    of this rank (graph mode: the warm-up runs the eager steps and the capture, the timed
    steps are replays).  Then, when `probe`, up to 5 more chunks run eagerly with the HIP-event
    probes around the kernel sites (per-kernel durations for the roofline; events cannot
    time kernels inside a replayed graph) -- untimed for the headline value.  Returns a dict
    (seconds = max over ranks)."""
    import nn as snn
    import optim
    import samplernn_hip as H
    from trainer import Trainer
    T, L = T_SEQ, 64
    m, pred = make_model(dtype)
    pred = pred.to(dev)
    sync = dist_mod.GradAllReduce(overlap_groups=dist_mod.readiness_groups(pred)) \
        if dist_mod.world() > 1 or os.environ.get('SRNN_DP_FORCE', '0') == '1' else None
    opt = optim.gradient_clipping(torch.optim.Adam(pred.parameters(), lr=1e-3), grad_sync=sync)
    n_probe = min(steps, 5) if probe else 0
    batches = gpu_batches(synth_batches(rows, T, L, warmup + steps + n_probe,
                                        dist_mod.rank() * rows), dev)
    tr = Trainer(pred, snn.sequence_nll_loss_bits, opt, batches[:warmup], True, None)
    log_ = _LossLog()
    tr.register_plugin(log_)
    tr.train()                              # warm-up chunks (ends with the failure check)
    torch.cuda.synchronize()
    dist_mod.barrier()
    torch.cuda.synchronize()
    tr.dataset = batches[warmup:warmup + steps]
    tr.enqueue_s = 0.0
    g0 = tr.graph_steps
    t0 = time.perf_counter()
    tr.train()                              # the timed chunks
    torch.cuda.synchronize()
    dist_mod.barrier()
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    enq = tr.enqueue_s
    replayed = tr.graph_steps - g0
    losses = [float(v) for v in log_.values]
    sites, eager_ms, eager_enq = {}, None, None
    if n_probe:
        tr.dataset = batches[warmup + steps:]
        tr.enqueue_s = 0.0
        H.ROOF_EVENTS = {}
        t1 = time.perf_counter()
        tr.train()
        torch.cuda.synchronize()
        eager_ms = (time.perf_counter() - t1) / n_probe * 1e3
        eager_enq = tr.enqueue_s / n_probe * 1e3
        ev, H.ROOF_EVENTS = H.ROOF_EVENTS, None
        for site, lst in (ev or {}).items():
            ms = sum(a.elapsed_time(b) for a, b, _ in lst) / n_probe
            work = sum(w for _, _, w in lst) / n_probe
            sites[site] = (ms, work, len(lst) // n_probe)
    dt = dist_mod.max_over_ranks(dt, dev)
    res = {'seconds': dt, 'ms_per_step': dt / steps * 1e3,
           'enqueue_ms_per_step': enq / steps * 1e3, 'graph_replays': replayed,
           'eager_ms_per_step': eager_ms, 'eager_enqueue_ms_per_step': eager_enq,
           'losses': losses[:warmup + steps], 'sites': sites, 'rows': rows}
    del tr, opt, pred, m, batches
    torch.cuda.empty_cache()
    return res


def tbptt_summary(r, N, dtype_peak, label):
    samples = N * r['rows'] * T_SEQ
    out = {'value': round(samples / (r['ms_per_step'] * 1e-3), 1), 'unit': 'samples/s',
           'ms_per_step': round(r['ms_per_step'], 3),
           'tbptt_steps_per_s': round(1e3 / r['ms_per_step'], 3),
           'rows_per_gpu': r['rows'], 'global_batch': N * r['rows'],
           'host_enqueue_ms_per_step': round(r['enqueue_ms_per_step'], 3),
           'graph_replays': r['graph_replays'],
           'eager_ms_per_step': r['eager_ms_per_step'] and round(r['eager_ms_per_step'], 3),
           'eager_host_enqueue_ms_per_step': r['eager_enqueue_ms_per_step'] and
           round(r['eager_enqueue_ms_per_step'], 3),
           'final_loss': round(r['losses'][-1], 4), 'workload': label}
    flops = step_mfma_flops(r['rows'])
    ach = flops / (r['ms_per_step'] * 1e-3) / 1e12
    out['step_mfma'] = {'flop_per_step': flops, 'achieved': round(ach, 1), 'peak': dtype_peak,
                        'unit': 'TFLOP/s', 'frac': round(ach / dtype_peak, 4)}
    return out


def kernels_block(r, dtype_peak):
    ks = {}
    for site, (ms, work, launches) in r['sites'].items():
        e = site_roofline(site, ms, work, dtype_peak)
        e.update({'ms_per_step': round(ms, 4), 'launches_per_step': launches,
                  'work_per_step': work})
        ks[site] = e
    return ks


def _pmc_file(pattern):
    """(bytes, source) from the newest committed rocprofv3 PMC pass matching pattern
    (profiles/r*_pmc_...txt: `avg_step_bytes` = 2 x FETCH_SIZE + WRITE_SIZE per step, gfx950
    FETCH correction per MI355X_MICROARCH.md) whose `csrc_hash` line equals the hash of the
    HIP sources this run's library is built from (samplernn_hip.csrc_hash); (None, reason)
    when no pass was taken on these kernels."""
    import glob
    import samplernn_hip as H
    want = H.csrc_hash()
    seen = []
    for path in sorted(glob.glob(os.path.join(ROOT, 'profiles', pattern)), reverse=True):
        b, h = None, None
        try:
            for line in open(path):
                f = line.split()
                if len(f) == 2 and f[0] == 'avg_step_bytes':
                    b = int(f[1])
                elif len(f) == 2 and f[0] == 'csrc_hash':
                    h = f[1]
        except (OSError, ValueError):
            continue
        name = os.path.basename(path)
        if b is not None and h == want:
            return b, '%s (csrc %s)' % (name, h)
        seen.append('%s at csrc %s' % (name, h))
    return None, 'no PMC pass at csrc %s%s' % (want, (' (stale: %s)' % ', '.join(seen))
                                              if seen else '')


def pmc_traffic(site, rows):
    """HBM bytes per step of a probed site (tools/pmc_site.sh), attributed to HEAD's kernels."""
    return _pmc_file('r*_pmc_%s_b%d.txt' % (site, rows))


def gru_sweep_roofline(dev, B=128, D=1024, Fr=64, reps=5):
    """MFMA utilisation of the recurrence's hidden x hidden products (the persistent XCD-grouped
    sweeps, gru_xcd.hip) in isolation: the bottom tier's forward and backward sweep at the
    TBPTT step's shape (bf16, B rows, Fr frames), HIP events on their stream; flop = Fr x 2 x B
    x 3D x D per sweep.  Latency-bound: one hand-off of h (dgh) per step."""
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
    res.update({'bound': 'latency (one hand-off of h / dgh per step)', 'unit': 'TFLOP/s',
                'peak': MI355X_BF16_TFLOPS,
                'kernel': 'gru_xcd_fwd/bwd_kernel in isolation, bottom tier B=%d D=%d %d frames'
                          % (B, D, Fr)})
    return res


def run_gen(dev, n_seqs, n_cond, dtype, frame_sizes=(16, 4), cond_dim=43, row0=0):
    """One timed Generator call over this rank's rows [row0, row0 + n_seqs); returns
    (seconds, algorithmic weight elements read per generation step: the sample-level MLP
    every step, tier k once per nfs_k steps)."""
    import model as M
    m, _ = make_model(dtype, seed=4242, frame_sizes=frame_sizes, cond_dim=cond_dim)
    m = m.to(dev)
    w_step = sum(p.numel() for p in m.sample_level_mlp.parameters()) + sum(
        sum(p.numel() for p in t.parameters()) / t.n_frame_samples for t in m.frame_level_rnns)
    cond = torch.rand(row0 + n_seqs, n_cond, cond_dim,
                      generator=torch.Generator().manual_seed(1))[row0:]
    spk = (np.arange(n_seqs) + row0) % 6
    gen = M.Generator(m, True)
    # warm-up (graph capture, kernel attributes) on a short run
    gen(n_seqs, 0, cond[:, :4], spk, sampler='philox', seed=5)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    gen(n_seqs, 0, cond, spk, sampler='philox', seed=5, row_offset=row0)
    torch.cuda.synchronize()
    return time.perf_counter() - t0, w_step


def gen_traffic(kind='gen'):
    """HBM bytes per generation step of a generation line (kind gen / gen_fp32 / gen_e /
    gen_e_fp32: B = 128, D = 1024) from the committed rocprofv3 PMC passes (tools/pmc_gen.sh:
    FETCH_SIZE kB x 2 + WRITE_SIZE kB over every dispatch of the loop's kernels / samples
    generated), attributed to HEAD's kernels."""
    return _pmc_file('r*_pmc_%s.txt' % kind)


def host_cores():
    """The host CPUs this process may use: the CPU affinity mask, capped by the cgroup's CPU
    quota (cpu.max) and by OMP_NUM_THREADS when set -- on the GPU box os.cpu_count() reports
    the whole machine, of which one GPU's job gets a share (the box sets OMP_NUM_THREADS to
    it).  `usable` is what the CPU baseline runs on (all of it)."""
    visible = os.cpu_count() or 1
    try:
        aff = len(os.sched_getaffinity(0))
    except (AttributeError, OSError):
        aff = visible
    quota = None
    for path in ('/sys/fs/cgroup/cpu.max',):
        try:
            q, per = open(path).read().split()[:2]
            if q != 'max':
                quota = max(1, int(int(q) / int(per)))
        except (OSError, ValueError):
            pass
    if quota is None:
        try:
            q = int(open('/sys/fs/cgroup/cpu/cpu.cfs_quota_us').read())
            per = int(open('/sys/fs/cgroup/cpu/cpu.cfs_period_us').read())
            if q > 0:
                quota = max(1, q // per)
        except (OSError, ValueError):
            pass
    usable = min(aff, quota) if quota else aff
    omp = os.environ.get('OMP_NUM_THREADS', '')
    if omp.isdigit() and int(omp) > 0:
        usable = min(usable, int(omp))      # the job's declared CPU share (16 per GPU box)
    return {'usable': usable, 'os_cpu_count': visible, 'affinity': aff, 'cgroup_quota': quota,
            'omp_num_threads': os.environ.get('OMP_NUM_THREADS')}


def cpu_baseline(seconds_budget=30.0):
    """The oracle (torch-CPU restatement of the reference, validated against the reference's
    timing here: profiles/r03_oracle_vs_reference.txt) on the host cores: a bounded TBPTT
    sample at configs[1]'s batch (B = 128 rows x T = 1024) and a bounded generation sample at
    configs[2]'s (128 utterances x 4 top-tier frames = 256 steps)."""
    sys.path.insert(0, os.path.join(ROOT, 'oracle'))
    import samplernn_oracle as O
    hc = host_cores()
    threads = hc['usable']
    torch.set_num_threads(threads)
    m, pred = make_model(torch.float32)
    sd = {k: v.detach().clone() for k, v in pred.state_dict().items()}
    cfg = dict(frame_sizes=[16, 4], n_rnn=1, dim=1024, q_levels=256, weight_norm=False,
               cond_dim=43, spk_dim=6)
    om = O.from_state_dict(cfg, sd)
    names = [k for k, p in pred.named_parameters()]
    opt = O.OracleAdam([om.p[k] for k in names], lr=1e-3)
    B = 128
    batches = synth_batches(B, 1024, 64, 3, 0)
    t0 = time.perf_counter()
    O.tbptt_step(om, opt, names, batches[0], return_grads=False)   # warm-up
    t_warm = time.perf_counter() - t0
    t0 = time.perf_counter()
    n = 0
    for b in batches[1:]:
        O.tbptt_step(om, opt, names, b, return_grads=False)
        n += 1
        if time.perf_counter() - t0 + t_warm > seconds_budget:
            break
    dt = time.perf_counter() - t0
    tb = {'value': round(n * B * 1024 / dt, 2), 'unit': 'samples/s', 'cores': threads,
          'kind': 'port', 'steps_per_s': round(n / dt, 4),
          'sample': '%d TBPTT step(s) of the oracle (torch-CPU fp32 restatement) at configs[1], '
                    'B=%d rows x T=1024, after 1 warm-up step, %d threads' % (n, B, threads)}
    # generation: 128 rows, 4 top-tier frames (256 steps) after a 1-frame warm-up
    gm = O.from_state_dict(cfg, {k: v.detach().clone() for k, v in
                                 make_model(torch.float32, seed=4242)[1].state_dict().items()})
    nb, nc = 128, 4
    cond = torch.rand(nb, nc, 43, generator=torch.Generator().manual_seed(1)).numpy()
    gm.generate(nb, cond[:, :1], np.arange(nb) % 6, None)
    t0 = time.perf_counter()
    gm.generate(nb, cond, np.arange(nb) % 6, None)      # Exp(1) per step, as multinomial
    dtg = time.perf_counter() - t0
    gen = {'value': round(nb * nc * 64 / dtg, 1), 'unit': 'samples/s', 'cores': threads,
           'kind': 'port', 'x_realtime': round(nb * nc * 64 / dtg / 16000, 3),
           'sample': 'oracle Generator loop (model.py:445-520 restated), 128 utterances x 256 '
                     'samples at configs[2] dims after a 64-sample warm-up, %d threads' % threads}
    tb['gen'] = gen
    tb['host_cores'] = hc
    return tb


def _free_port():
    import socket
    s = socket.socket(socket.AF_INET, socket.SOCK_STREAM)
    s.bind(('127.0.0.1', 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _die_with_parent():
    """preexec_fn of a rank: SIGKILL it if the launching process dies (a killed parent must
    not leave ranks waiting in a collective)."""
    import ctypes
    import signal
    try:
        ctypes.CDLL('libc.so.6', use_errno=True).prctl(1, signal.SIGKILL)   # PR_SET_PDEATHSIG
    except OSError:
        pass


def spawn_ranks(n, argv=None, env=None, poll_s=0.5, script=None):
    """`python bench.py --gpus N` outside torchrun: start N fresh child processes of this
    script, one per GPU, with the torchrun environment (RANK = LOCAL_RANK = r, WORLD_SIZE =
    LOCAL_WORLD_SIZE = N, MASTER_ADDR 127.0.0.1, a free MASTER_PORT); distributed.init pins
    each to cuda:LOCAL_RANK and opens the process group (RCCL unless SRNN_DIST_BACKEND says
    otherwise).  This process never touches a GPU and never execs: it forwards rank 0's
    stdout (the JSON line), lets every rank's stderr through, and returns non-zero -- after
    killing the other ranks -- as soon as any rank fails.  Returns the exit status."""
    import subprocess
    import threading
    argv = list(sys.argv[1:] if argv is None else argv)
    backend = (env or os.environ).get('SRNN_DIST_BACKEND', 'nccl')
    ndev = torch.cuda.device_count()          # does not initialise the GPU on this image
    if backend == 'nccl' and script is None and ndev < n:
        log('bench: --gpus %d needs %d visible GPUs for RCCL (one rank per GPU), %d visible; '
            'SRNN_DIST_BACKEND=gloo runs a rehearsal with ranks sharing GPUs' % (n, n, ndev))
        return 2
    port = _free_port()
    procs, out_lines = [], []
    for r in range(n):
        e = dict(os.environ if env is None else env)
        e.update({'RANK': str(r), 'LOCAL_RANK': str(r), 'WORLD_SIZE': str(n),
                  'LOCAL_WORLD_SIZE': str(n), 'GROUP_RANK': '0', 'MASTER_ADDR': '127.0.0.1',
                  'MASTER_PORT': str(port)})
        procs.append(subprocess.Popen(
            [sys.executable, script or os.path.abspath(__file__)] + argv, env=e,
            stdout=subprocess.PIPE if r == 0 else sys.stderr, preexec_fn=_die_with_parent,
            text=True))
    log('bench: %d ranks spawned (pids %s, master 127.0.0.1:%d)'
        % (n, ' '.join(str(p.pid) for p in procs), port))

    def pump():
        for line in procs[0].stdout:
            out_lines.append(line)
    reader = threading.Thread(target=pump, daemon=True)
    reader.start()
    rc = 0
    try:
        while True:
            codes = [p.poll() for p in procs]
            bad = [(r, c) for r, c in enumerate(codes) if c not in (None, 0)]
            if bad:
                rc = bad[0][1] if bad[0][1] > 0 else 128 - bad[0][1]
                log('bench: rank %d exited with %s; stopping the other ranks' % bad[0])
                break
            if all(c == 0 for c in codes):
                break
            time.sleep(poll_s)
    finally:
        for p in procs:
            if p.poll() is None:
                p.terminate()
        for p in procs:
            try:
                p.wait(timeout=20)
            except subprocess.TimeoutExpired:
                p.kill()
                p.wait()
        reader.join(timeout=10)
    for line in out_lines:
        sys.stdout.write(line)
    sys.stdout.flush()
    return rc


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--gpus', type=int, default=1)
    ap.add_argument('--steps', type=int, default=10)
    ap.add_argument('--warmup', type=int, default=3)
    ap.add_argument('--batch', type=int, default=None,
                    help='rows per GPU (default: configs[3], global 512 / N, strong scaling)')
    ap.add_argument('--dtype', default='bf16', choices=['bf16', 'fp32'])
    ap.add_argument('--gen-dtype', default='bf16', choices=['bf16', 'fp32'])
    ap.add_argument('--no-gen-fp32', action='store_true')
    ap.add_argument('--no-gen-e', action='store_true')
    ap.add_argument('--gen-seqs', type=int, default=128, help='utterances per GPU')
    ap.add_argument('--gen-cond', type=int, default=750)
    ap.add_argument('--no-gen', action='store_true')
    ap.add_argument('--no-cpu', action='store_true')
    ap.add_argument('--no-extra', action='store_true', help='skip config_b / weak_64 lines')
    args = ap.parse_args()

    if args.gpus > 1 and 'WORLD_SIZE' not in os.environ:
        # not under torchrun: this process touches no GPU and runs N ranks as children
        sys.exit(spawn_ranks(args.gpus))

    import distributed as D
    D.init()
    dev = torch.device('cuda', D.device_index())
    torch.cuda.set_device(dev)
    N = D.world()
    pg = {'backend': None, 'world_size': 1}
    if torch.distributed.is_available() and torch.distributed.is_initialized():
        N = torch.distributed.get_world_size()
        pg = {'backend': torch.distributed.get_backend(), 'world_size': N}
    if N != args.gpus:
        log('warning: --gpus %d but the process group has %d rank(s)' % (args.gpus, N))
    dtype = torch.bfloat16 if args.dtype == 'bf16' else torch.float32
    peak = MI355X_BF16_TFLOPS if args.dtype == 'bf16' else MI355X_FP32_TFLOPS
    strong = args.batch is None
    rows = GLOBAL_B // N if strong else args.batch
    if strong and GLOBAL_B % N:
        raise SystemExit('global batch %d not divisible by %d ranks' % (GLOBAL_B, N))

    main_r = run_tbptt(dev, D, rows, args.steps, args.warmup, dtype)
    log('tbptt %d rows/GPU: %.2f ms/step (host enqueue %.2f ms/step, %d graph replays; eager '
        '%s ms/step), losses %s' % (
        rows, main_r['ms_per_step'], main_r['enqueue_ms_per_step'], main_r['graph_replays'],
        main_r['eager_ms_per_step'],
        ['%.3f' % l for l in main_r['losses']]))
    label = ('configs[3]: TBPTT step, 3-tier SampleRNN dim1024 FS=[16,4] n_rnn=1 cond 43 spk 6, '
             'T=1024, global batch %d = %d rows/GPU x %d GPU, Trainer.train (fwd+bwd+%sclip+'
             'Adam)' % (N * rows, rows, N, 'all-reduce+' if N > 1 else ''))
    summ = tbptt_summary(main_r, N, peak, label)
    ks = kernels_block(main_r, peak)
    dom = max(ks, key=lambda k: ks[k]['ms_per_step']) if ks else None
    roof = None
    if dom:
        roof = dict(ks[dom])
        roof['traffic'], roof['traffic_source'] = pmc_traffic(dom, rows)
        roof['kernel'] = '%s; %.3f ms per step (%d launches; HIP events on the launching stream '\
                         'around each launch, over eager steps of the same run right after the '\
                         'timed graph replays)' % (SITE_NOTES.get(dom, dom), ks[dom]['ms_per_step'],
                                                   ks[dom]['launches_per_step'])
        roof['site'] = dom

    extra = {}
    if not args.no_extra:
        if N == 1 and not (not strong and rows == 128):
            r = run_tbptt(dev, D, 128, args.steps, args.warmup, dtype)
            extra['config_b'] = tbptt_summary(
                r, N, peak, 'configs[1]: the same step at B=128 rows on one GPU')
            extra['config_b']['kernels'] = kernels_block(r, peak)
            log('config_b: %.2f ms/step' % r['ms_per_step'])
        if N == 1 and args.dtype == 'bf16':
            # the same step with every GEMM on the hand-written kernels (hipBLASLt off):
            # the kernel-quality number for the hand-written path alone
            os.environ['SRNN_BLASLT'] = '0'
            try:
                r = run_tbptt(dev, D, rows, args.steps, args.warmup, dtype, probe=False)
            finally:
                del os.environ['SRNN_BLASLT']
            extra['handwritten_only'] = tbptt_summary(
                r, N, peak, 'the headline step with SRNN_BLASLT=0: every GEMM on the '
                'hand-written gemm3 / gemm2 / skinny kernels, no vendor library kernel')
            log('handwritten_only: %.2f ms/step' % r['ms_per_step'])
        if N > 1 and strong:
            # weak scaling beside the strong-scaling headline: each rank keeps the N = 1 line's
            # 512 rows (global batch 512 N), so per-GPU work is the headline's and only the
            # all-reduce is added (scaling efficiency = this value / (N x the N = 1 value))
            r = run_tbptt(dev, D, GLOBAL_B, args.steps, args.warmup, dtype, probe=False)
            extra['weak_512'] = tbptt_summary(
                r, N, peak, '512 rows per GPU x %d GPU (global batch %d, weak scaling)'
                % (N, GLOBAL_B * N))
            log('weak_512: %.2f ms/step' % r['ms_per_step'])
        if not (not strong and rows == 64) and not (strong and rows == 64):
            r = run_tbptt(dev, D, 64, args.steps, args.warmup, dtype)
            extra['weak_64'] = tbptt_summary(
                r, N, peak, '64 rows per GPU x %d GPU (configs[3]\'s 8-GPU share, weak scaling)'
                % N)
            log('weak_64: %.2f ms/step' % r['ms_per_step'])

    gru = None
    if args.dtype == 'bf16':
        gru = gru_sweep_roofline(dev, B=rows)

    def gen_line(dname, frame_sizes=(16, 4), cond_dim=43, n_cond=None, tag='3-tier dim1024 '
                 'FS=[16,4]'):
        gdt = torch.bfloat16 if dname == 'bf16' else torch.float32
        n_cond = n_cond or args.gen_cond
        L = int(np.prod(frame_sizes))
        t, W_step = run_gen(dev, args.gen_seqs, n_cond, gdt, frame_sizes, cond_dim,
                            row0=D.rank() * args.gen_seqs)
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
        line = {'value': round(gs, 1), 'unit': 'samples/s', 'x_realtime': round(gs / 16000, 1),
                'x_realtime_per_gpu': round(gs / 16000 / N, 1), 'dtype': dname,
                'seconds': round(t, 3), 'steps_per_s': round(steps_per_s, 1),
                'us_per_step': round(1e6 / steps_per_s, 2),
                'sample_loop': ('persistent (gen_mlp.hip, %d rows/group)' % rows_pg) if rows_pg
                               else 'per-sample kernels (hipGraph)',
                'config': {'workload': 'generate %s cond %d, %d utt x %d cond rows (%d samples) '
                                       'per GPU (rows %d..%d of %d), Philox sampler'
                                       % (tag, cond_dim, args.gen_seqs, n_cond, n_cond * L,
                                          D.rank() * args.gen_seqs,
                                          (D.rank() + 1) * args.gen_seqs - 1, N * args.gen_seqs)},
                'roofline': {'bound': 'hbm',
                             'achieved': round(bytes_step * steps_per_s / 1e9, 1),
                             'peak': MI355X_HBM_TBS * 1000, 'unit': 'GB/s',
                             'frac': round(bytes_step * steps_per_s / 1e9 /
                                           (MI355X_HBM_TBS * 1000), 4),
                             'traffic': None, 'traffic_source': 'no PMC pass for this line'}}
        if args.gen_seqs == 128:
            kind = ('gen' if tuple(frame_sizes) == (16, 4) else 'gen_e') + \
                ('' if dname == 'bf16' else '_fp32')
            line['roofline']['traffic'], line['roofline']['traffic_source'] = gen_traffic(kind)
        return line

    gen = gen_fp32 = gen_e = gen_e_fp32 = None
    if not args.no_gen:
        gen = gen_line(args.gen_dtype)
        if args.gen_dtype != 'fp32' and not args.no_gen_fp32:
            gen_fp32 = gen_line('fp32')       # the reference's precision (bit-replay tests)
        if not args.no_gen_e:
            # configs[4]: 4-tier + look-ahead conditioning (C = 86), 1024 utterances over 8
            # GPUs = 128 per GPU, 188 cond rows x 256 = 48,128 samples each
            gen_e = gen_line(args.gen_dtype, (16, 4, 4), 86, 188,
                             '4-tier dim1024 FS=[16,4,4] look-ahead')
            if args.gen_dtype != 'fp32' and not args.no_gen_fp32:
                gen_e_fp32 = gen_line('fp32', (16, 4, 4), 86, 188,
                                      '4-tier dim1024 FS=[16,4,4] look-ahead')

    cpu = None
    if D.rank() == 0 and N == 1 and not args.no_cpu:
        cpu = cpu_baseline()

    if D.rank() == 0:
        line = {'metric': METRIC, 'value': summ['value'], 'unit': 'samples/s',
                'n_gpus': N, 'steps': args.steps, 'warmup': args.warmup,
                'rccl_ranks': pg['world_size'] if pg['backend'] == 'nccl' else 0,
                'process_group': pg,
                'ms_per_step': summ['ms_per_step'], 'higher_is_better': True,
                'scaling': 'strong' if strong else 'weak',
                'vs_baseline': None, 'dtype': args.dtype, 'data': 'synthetic',
                'config': {'workload': label, 'global_batch': N * rows, 'seq_len': T_SEQ,
                           'rows_per_gpu': rows, 'parallelism': 'dp%d' % N},
                'tbptt_steps_per_s': summ['tbptt_steps_per_s'],
                'host_enqueue_ms_per_step': summ['host_enqueue_ms_per_step'],
                'graph_replays': summ['graph_replays'],
                'eager_ms_per_step': summ['eager_ms_per_step'],
                'eager_host_enqueue_ms_per_step': summ['eager_host_enqueue_ms_per_step'],
                'roofline': roof, 'kernels': ks, 'step_mfma': summ['step_mfma'],
                'cpu_baseline': cpu, 'gen': gen, 'gen_fp32': gen_fp32,
                'gen_config_e': gen_e, 'gen_config_e_fp32': gen_e_fp32, 'gru_sweep': gru,
                'final_loss': summ['final_loss']}
        line.update(extra)
        print(json.dumps(line), flush=True)
    D.barrier()


if __name__ == '__main__':
    main()
