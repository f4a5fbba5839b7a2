"""SURVEY §8d check: the oracle (torch-CPU restatement, oracle/samplernn_oracle.py) must time
within +-15 % of the reference itself at the same thread count, so that timing the oracle on
the GPU box's host cores stands in for the reference's CPU path (which cannot travel there).

Runs HERE only (imports the reference from /root/reference through make_golden's harness):
configs[1] / [2] dims (3-tier, dim 1024, FS [16, 4], cond 43, 6 speakers), 8 threads,
  * one TBPTT step (forward, NLL, backward, clip, Adam) at B = 1 (the reference Predictor
    only runs at B = 1, model.py:209), T = 1024;
  * generation of 128 rows x 64 samples (one top-tier frame) after a 64-sample warm-up.
Writes profiles/r03_oracle_vs_reference.txt.

Usage: python tests/golden/time_oracle_vs_reference.py
"""
import os
import sys
import time

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, HERE)
import make_golden as MG  # noqa: E402  (imports the reference; chdir to a scratch dir)

torch = MG.torch
sys.path.insert(0, os.path.join(ROOT, 'oracle'))
import samplernn_oracle as O  # noqa: E402
import recipe  # noqa: E402
import numpy as np  # noqa: E402

torch.set_num_threads(8)
cfg = recipe.CONFIGS['big']
w = recipe.make_weights(cfg, 16)
lines = []


def best(fn, reps):
    ts = []
    for _ in range(reps):
        t0 = time.perf_counter()
        fn()
        ts.append(time.perf_counter() - t0)
    return min(ts)


# ---- TBPTT step at B = 1
x, reset, tgt, cond, spk = MG.make_chunks(cfg, 1, 1024, 1, 7)[1][0]
m_ref, pred_ref = MG.build_ref(cfg, w)
opt_ref = MG.ref_optim.gradient_clipping(MG._Adam(pred_ref.parameters(), lr=1e-3))


def ref_step():
    opt_ref.zero_grad()

    def closure():
        out = pred_ref(torch.from_numpy(x), True, torch.from_numpy(cond), torch.from_numpy(spk),
                       None, 0)
        loss = MG.ref_nn.sequence_nll_loss_bits(out, torch.from_numpy(tgt))
        loss.backward()
        return loss
    opt_ref.step(closure)


om = O.from_state_dict(cfg, w)
names = list(w.keys())
opt_o = O.OracleAdam([om.p[k] for k in names], lr=1e-3)


def oracle_step():
    O.tbptt_step(om, opt_o, names, (torch.from_numpy(x), True, torch.from_numpy(tgt),
                                    torch.from_numpy(cond), torch.from_numpy(spk)),
                 return_grads=False)


ref_step()
oracle_step()
t_ref = best(ref_step, 5)
t_orc = best(oracle_step, 5)
lines.append('tbptt B=1 T=1024 (8 threads): reference %.3f s  oracle %.3f s  ratio %.3f'
             % (t_ref, t_orc, t_orc / t_ref))

# ---- generation, 128 rows x 64 samples
n, nc = 128, 1
gcond = recipe.synth_cond((nc, cfg['cond_dim']), 3)
m_g, _ = MG.build_ref(cfg, w)
gen_ref = MG.ref_model.Generator(m_g, False)
noise = torch.empty(64 * nc, n, 256).exponential_(1)
og = O.from_state_dict(cfg, w)
devnull = open(os.devnull, 'w')


def ref_gen():
    so = sys.stdout
    sys.stdout = devnull
    try:
        with torch.no_grad():
            gen_ref(n, 0, gcond, 2)
    finally:
        sys.stdout = so


def oracle_gen():
    og.generate(n, gcond, 2, None)          # Exp(1) drawn per step, as multinomial does


ref_gen()
oracle_gen()
g_ref = best(ref_gen, 2)
g_orc = best(oracle_gen, 2)
lines.append('generate 128 rows x 64 samples (8 threads): reference %.3f s (%.0f samples/s)  '
             'oracle %.3f s (%.0f samples/s)  ratio %.3f'
             % (g_ref, n * 64 / g_ref, g_orc, n * 64 / g_orc, g_orc / g_ref))
lines.append('within +-15 %%: tbptt %s, generate %s' % (
    abs(t_orc / t_ref - 1) <= 0.15, abs(g_orc / g_ref - 1) <= 0.15))
out = os.path.join(ROOT, 'profiles', 'r03_oracle_vs_reference.txt')
with open(out, 'w') as f:
    f.write('# tests/golden/time_oracle_vs_reference.py (this container, %d CPUs, torch %s)\n'
            % (os.cpu_count(), torch.__version__))
    f.write('\n'.join(lines) + '\n')
print('\n'.join(lines))
