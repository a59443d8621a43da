"""bench.py host logic (no GPU): the --gpus N launcher and the CPU-baseline core grant."""
import os
import subprocess
import sys

import pytest

from conftest import REPO

sys.path.insert(0, REPO)
import bench  # noqa: E402


def test_launcher_spawns_n_ranks():
    cmd = bench.launch_command(['--gpus', '4', '--steps', '2'], {}, n_devices=8, gpus=4)
    assert cmd[:3] == [sys.executable, '-m', 'torch.distributed.run']
    assert cmd[cmd.index('--nproc-per-node') + 1] == '4'
    assert cmd[cmd.index('--master-addr') + 1] == '127.0.0.1'
    assert cmd[-3:] == ['--gpus', '4', '--steps', '2'][-3:]
    assert os.path.samefile(cmd[cmd.index('--gpus') - 1], os.path.join(REPO, 'bench.py'))


def test_launcher_noop_inside_a_rank_or_single_gpu():
    assert bench.launch_command(['--gpus', '1'], {}, 8, 1) is None
    assert bench.launch_command(['--gpus', '2'], {'WORLD_SIZE': '2'}, 8, 2) is None
    with pytest.raises(SystemExit):  # an outer launcher with a different world size
        bench.launch_command(['--gpus', '4'], {'WORLD_SIZE': '2'}, 8, 4)


def test_launcher_refuses_more_ranks_than_gpus():
    with pytest.raises(SystemExit, match='only 1 GPU'):
        bench.launch_command(['--gpus', '2'], {}, 1, 2)
    # the one-GPU rehearsal shares cuda:0 between ranks
    assert bench.launch_command(['--gpus', '2'], {'LDDL_BENCH_SHARE_DEVICE': '1'}, 1, 2)


def test_launcher_end_to_end_without_gpus():
    """`python bench.py --gpus 2` on a box with no GPU fails loudly instead of running one rank."""
    env = dict(os.environ)
    env.pop('WORLD_SIZE', None)
    env.pop('LDDL_BENCH_SHARE_DEVICE', None)
    r = subprocess.run([sys.executable, os.path.join(REPO, 'bench.py'), '--gpus', '2'], env=env,
                       stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True, timeout=300)
    assert r.returncode != 0 and 'visible' in r.stderr


def test_granted_cores():
    cores, how = bench.granted_cores()
    assert 1 <= cores <= len(os.sched_getaffinity(0))
    assert 'sched_getaffinity' in how and 'os.cpu_count()' in how


def test_pmc_json_matches_actual_batch_and_template_names():
    """The committed PMC passes are found by the batch's actual byte count and the planner's
    template instantiation is found by its base name (bench.py `traffic` / `issue_roofline`)."""
    kernels, src, meta = bench.load_pmc((10_000_000_000, 10_000_001_451))
    assert src is not None and kernels and set(meta) == {'build_id', 'git_head'}
    plan = bench.pmc_entry(kernels, 'plan_replay_kernel')
    assert plan.get('SQ_INSTS_SALU') and plan.get('hbm_bytes_per_launch')
    assert bench.pmc_entry(kernels, 'tokenize_batch_kernel').get('SQ_INSTS_VALU')
    assert bench.pmc_entry(kernels, 'no_such_kernel') == {}


def test_partition_prefix():
    """c4_exchange's sub-batch: whole leading partitions within the byte budget, at least one."""
    import types
    import numpy as np
    sent_off = np.arange(0, 1001, 10, dtype=np.int64)       # 100 sentences of 10 bytes
    doc_sent_off = np.arange(0, 101, 2, dtype=np.int64)     # 50 documents of 2 sentences
    corp = types.SimpleNamespace(sent_off=sent_off, doc_sent_off=doc_sent_off)
    part = np.arange(0, 51, 5, dtype=np.int64)              # 10 partitions of 100 bytes
    assert bench.partition_prefix(corp, part, 350) == 3
    assert bench.partition_prefix(corp, part, 400) == 4
    assert bench.partition_prefix(corp, part, 10) == 1
    assert bench.partition_prefix(corp, part, 10 ** 9) == 10


@pytest.mark.gpu
def test_bench_c4_exchange_subline_two_ranks():
    """`bench.py --gpus 2` in the one-GPU rehearsal (LDDL_BENCH_SHARE_DEVICE=1: two ranks on
    cuda:0, gloo through host tensors): the C2 line carries the c4_exchange sub-line, with rows
    moved between the ranks and every bin's shards within one row."""
    import json
    env = dict(os.environ, LDDL_BENCH_SHARE_DEVICE='1')
    env.pop('WORLD_SIZE', None)
    r = subprocess.run([sys.executable, os.path.join(REPO, 'bench.py'), '--gpus', '2', '--steps', '1',
                        '--warmup', '0', '--batch-bytes', '60000000', '--exchange-bytes', '40000000',
                        '--no-alt-rng', '--no-segmented-line', '--no-extra-lines'],
                       env=env, stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-3000:]
    line = json.loads([x for x in r.stdout.splitlines() if x.startswith('{')][-1])
    assert line['n_gpus'] == 2
    ex = line['c4_exchange']
    assert ex['backend'] == 'gloo' and ex['num_shards'] == 16
    assert ex['moved_rows'] > 0 and ex['rows'] > ex['moved_rows']
    assert ex['shard_counts_spread'] <= 1
    assert ex['exchange_ms'] >= 0
