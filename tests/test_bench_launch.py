"""bench.py --gpus N starts its own ranks: with no RANK in the environment
the parent makes no GPU call, runs a child torch.distributed.run on 127.0.0.1 and relays rank 0's
JSON line. CPU: the launcher with a stub rank script (gloo, world size 2). GPU: the real bench at
--gpus 2 on the one-GPU box (both ranks on device 0, gloo coordination): n_gpus 2, a cpu_baseline
and zero parity mismatches summed over both ranks' shards."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

STUB = '''
import json, os, sys
import torch.distributed as dist
dist.init_process_group('gloo')
import torch
t = torch.tensor([float(dist.get_rank() + 1)])
dist.all_reduce(t)
if dist.get_rank() == 0:
    print('banner line a native library might print')
    print(json.dumps({'world': dist.get_world_size(), 'sum': float(t[0]), 'argv': sys.argv[1:]}))
dist.destroy_process_group()
'''


def test_self_launch_relays_rank0_line(tmp_path):
    stub = tmp_path / 'rank.py'
    stub.write_text(STUB)
    code = ('import sys; sys.path.insert(0, %r); import bench; '
            'sys.exit(bench.self_launch(2, ["--steps", "3"], script=%r))' % (ROOT, str(stub)))
    p = subprocess.run([sys.executable, '-c', code], capture_output=True, text=True, timeout=300, cwd=ROOT)
    assert p.returncode == 0, p.stderr[-3000:]
    lines = p.stdout.strip().splitlines()
    assert len(lines) == 1, p.stdout
    out = json.loads(lines[0])
    assert out == {'world': 2, 'sum': 3.0, 'argv': ['--steps', '3']}


def test_external_launch_must_match_gpus():
    env = dict(os.environ, RANK='0', WORLD_SIZE='2', LOCAL_RANK='0', MASTER_PORT='1', MASTER_ADDR='127.0.0.1')
    p = subprocess.run([sys.executable, 'bench.py', '--gpus', '4'], capture_output=True, text=True, timeout=300,
                       cwd=ROOT, env=env)
    assert p.returncode != 0 and 'WORLD_SIZE=2 but --gpus 4' in p.stderr


@pytest.mark.gpu
def test_bench_two_ranks_on_one_gpu():
    cmd = [sys.executable, 'bench.py', '--gpus', '2', '--steps', '3', '--warmup', '1', '--files-per-gpu', '40000',
           '--extra-configs', '3,5', '--extra-files-per-gpu', '20000', '--no-extras', '--cpu-seconds', '1']
    p = subprocess.run(cmd, capture_output=True, text=True, timeout=900, cwd=ROOT)
    assert p.returncode == 0, p.stderr[-4000:]
    line = json.loads(p.stdout.strip().splitlines()[-1])
    assert line['n_gpus'] == 2 and line['config']['global_files'] == 80000
    assert line['extras']['process_group']['world_size'] == 2
    assert line['cpu_baseline'] and line['cpu_baseline']['value'] > 0
    assert line['parity']['mismatches'] == 0 and line['parity']['ranks_checked'] == 2
    # the host gather: both ranks' results in rank 0's shared host buffer, checked
    ex = line['extras']
    assert ex['host_gather_mismatches'] == 0 and ex['host_gather_checked'] is True, ex
    assert ex['gather_winner'] == 'host' and 'no RCCL' in ex['gather_note'] and ex['host_gather_ms'] > 0
    for tag in ('3', '3-top1', '3-allpairs', '5'):
        rec = line['extras']['configs'][tag]
        assert rec['global_files'] == 40000 and rec['parity']['mismatches'] == 0, (tag, rec)
        assert rec['cpu_baseline']['value'] > 0


@pytest.mark.gpu
def test_bench_abi_sharded_leg_three_contexts():
    """--shard-mode abi: dice_match_sharded_confidence over 3 contexts (all on device 0 of the test
    box), host and device gathers timed, results equal to the resident batch's."""
    cmd = [sys.executable, 'bench.py', '--steps', '3', '--warmup', '1', '--files-per-gpu', '50000',
           '--extra-configs=', '--no-extras', '--no-cpu-baseline', '--shard-mode', 'abi', '--abi-contexts', '3']
    p = subprocess.run(cmd, capture_output=True, text=True, timeout=900, cwd=ROOT)
    assert p.returncode == 0, p.stderr[-4000:]
    rec = json.loads(p.stdout.strip().splitlines()[-1])['extras']['abi_sharded']
    assert rec['contexts'] == 3 and rec['devices'] == [0, 0, 0] and rec['files'] == 50000
    for mode in ('host', 'device'):
        assert rec[mode]['mismatches'] == 0 and rec[mode]['files_per_s'] > 0, rec
    # one device: no peer path exercised, and no gather winner claimed from same-device timings
    assert rec['host']['dice_last_gather_peer'] == -1 and rec['device']['dice_last_gather_peer'] == -1
    assert rec['winner'] is None and 'distinct device' in rec['winner_reason']


def test_config3_traffic_file_per_entry_point():
    """Config 3's roofline.traffic comes from the PMC file of the entry point measured: '3' through
    dice_batch_match_confidence (pmc_config3.json), '3-top1' through dice_batch_match
    (pmc_config3_top1.json), '3-allpairs' on the postings kernels (pmc_config3_post.json)."""
    import sys
    sys.path.insert(0, ROOT)
    import bench
    from types import SimpleNamespace as R
    assert bench.traffic_variant(3, R(match_kernel=4, confidence=True)) == ''
    assert bench.traffic_variant(3, R(match_kernel=4, confidence=False)) == '_top1'
    assert bench.traffic_variant(3, R(match_kernel=3, confidence=False)) == '_post'
    assert bench.traffic_variant(2, R(match_kernel=1, confidence=False)) == ''
    for name in ('pmc_config3.json', 'pmc_config3_top1.json', 'pmc_config3_post.json'):
        assert os.path.exists(os.path.join(ROOT, 'profiles', name)), name
