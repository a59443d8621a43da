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
