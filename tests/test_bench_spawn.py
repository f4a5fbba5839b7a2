"""bench.py --gpus N outside torchrun: the parent spawns N ranks itself (verdict r05 #1).

CPU tests of bench.spawn_ranks with stand-in rank scripts (no GPU): the children get the
torchrun environment, rank 0's stdout is forwarded, and a failing rank stops the others and
makes the parent exit non-zero.  distributed.device_share counts ranks per physical GPU.
"""
import json
import os
import sys
import textwrap
import time

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, 'jalil-saboorizadeh-multi-speaker-neural-vocoder_amd'))


def _script(tmp_path, body):
    p = tmp_path / 'rank.py'
    p.write_text(textwrap.dedent(body))
    return str(p)


def test_spawn_ranks_sets_torchrun_env_and_forwards_rank0(tmp_path, capfd):
    import bench
    s = _script(tmp_path, """
        import json, os, sys
        keys = ('RANK', 'LOCAL_RANK', 'WORLD_SIZE', 'LOCAL_WORLD_SIZE', 'MASTER_ADDR',
                'MASTER_PORT')
        env = {k: os.environ[k] for k in keys}
        if env['RANK'] == '0':
            print(json.dumps(env))
        else:
            print('rank %s' % env['RANK'], file=sys.stderr)
    """)
    rc = bench.spawn_ranks(3, argv=['--gpus', '3'], script=s, poll_s=0.05)
    assert rc == 0
    out = capfd.readouterr().out.strip().splitlines()
    assert len(out) == 1
    env = json.loads(out[0])
    assert env['RANK'] == '0' and env['LOCAL_RANK'] == '0'
    assert env['WORLD_SIZE'] == '3' and env['LOCAL_WORLD_SIZE'] == '3'
    assert env['MASTER_ADDR'] == '127.0.0.1' and int(env['MASTER_PORT']) > 0


def test_spawn_ranks_failing_rank_stops_the_rest(tmp_path):
    import bench
    s = _script(tmp_path, """
        import os, sys, time
        if os.environ['RANK'] == '1':
            sys.exit(3)
        time.sleep(120)          # would wait forever in a collective
    """)
    t0 = time.time()
    rc = bench.spawn_ranks(2, argv=[], script=s, poll_s=0.05)
    assert rc == 3
    assert time.time() - t0 < 60


def test_spawn_ranks_refuses_more_rccl_ranks_than_gpus():
    import bench
    env = dict(os.environ)
    env.pop('SRNN_DIST_BACKEND', None)
    # no GPU in this container: RCCL ranks cannot be placed, and nothing is started
    import torch
    if torch.cuda.device_count() >= 2:
        pytest.skip('GPUs visible')
    assert bench.spawn_ranks(2, argv=[], env=env) == 2


def test_device_share_counts_ranks_on_the_same_card():
    import distributed as D
    a = ('host0', '0000:05:00', 'uuid-a')
    b = ('host0', '0000:15:00', 'uuid-b')
    c = ('host1', '0000:05:00', 'uuid-c')
    # dedicated GPUs (per-rank *_VISIBLE_DEVICES: every process sees one device 0)
    assert D.device_share([a, b, c], a) == 1
    # two ranks on one card (the one-GPU rehearsal)
    assert D.device_share([a, a, b], a) == 2
    assert D.device_share([list(a), list(a)], a) == 2


def test_host_cores_reports_the_share():
    import bench
    hc = bench.host_cores()
    assert 1 <= hc['usable'] <= hc['affinity'] <= hc['os_cpu_count']
