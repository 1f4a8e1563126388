"""N>1 path on CPU: world_size-2 gloo process group running the same sharding / broadcast / timing code
bench.py runs over RCCL (spef_amd/shard.py)."""
import hashlib
import os
import socket
import tempfile

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp


def _free_port():
    with socket.socket() as s:
        s.bind(('127.0.0.1', 0))
        return s.getsockname()[1]


def _worker(rank, world, port, out_dir):
    import sys
    here = os.path.dirname(os.path.abspath(__file__))
    repo = os.path.dirname(here)
    sys.path[:0] = [repo, os.path.join(repo, 'spacecraft-pose-estimation-framework_amd')]
    from bench import synth_frames
    from spef_amd import blob as Bl
    from spef_amd.arch import mobilenet_v2
    from spef_amd.shard import broadcast_blob, gather_poses, max_over_ranks, shard_range
    from spef_amd.weights import synthetic_state_dict

    dist.init_process_group('gloo', init_method=f'tcp://127.0.0.1:{port}', rank=rank, world_size=world)
    dev = torch.device('cpu')
    blob = Bl.pack(synthetic_state_dict(mobilenet_v2(), seed=1001)) if rank == 0 else None
    got = broadcast_blob(blob, dev)
    digest = hashlib.sha256(got.numpy().tobytes()).hexdigest()

    n_frames = 5                                  # ragged: ranks get 3 and 2 frames
    a, b = shard_range(n_frames, rank, world)
    fr = synth_frames(b - a, 32, 48, a)
    t = max_over_ranks(0.5 + rank, dev)           # rank 1 is the slow one

    ori = torch.full((b - a, 4), float(rank)) + torch.arange(b - a)[:, None].float()
    pos = torch.full((b - a, 3), 10.0 * rank)
    go, gp = gather_poses(ori, pos)
    np.savez(os.path.join(out_dir, f'r{rank}.npz'), digest=digest, a=a, b=b, frames=fr, t=t,
             go=go if go is not None else np.zeros(0), gp=gp if gp is not None else np.zeros(0))
    dist.barrier()
    dist.destroy_process_group()


@pytest.fixture(scope='module')
def ranks():
    world = 2
    with tempfile.TemporaryDirectory() as d:
        mp.spawn(_worker, args=(world, _free_port(), d), nprocs=world, join=True)
        yield [dict(np.load(os.path.join(d, f'r{r}.npz'))) for r in range(world)]


def test_blob_broadcast_identical(ranks):
    from spef_amd import blob as Bl
    from spef_amd.arch import mobilenet_v2
    from spef_amd.weights import synthetic_state_dict
    want = hashlib.sha256(Bl.pack(synthetic_state_dict(mobilenet_v2(), seed=1001))).hexdigest()
    assert all(str(r['digest']) == want for r in ranks)


def test_shards_partition_the_frames(ranks):
    from bench import synth_frames
    assert [(int(r['a']), int(r['b'])) for r in ranks] == [(0, 3), (3, 5)]
    # frames depend on (seed, global index) only: the shards concatenate to the single-process frames
    whole = synth_frames(5, 32, 48, 0)
    np.testing.assert_array_equal(np.concatenate([r['frames'] for r in ranks]), whole)


def test_time_is_max_over_ranks(ranks):
    assert all(float(r['t']) == 1.5 for r in ranks)


def test_gather_poses_rank_order(ranks):
    go, gp = ranks[0]['go'], ranks[0]['gp']
    assert go.shape == (5, 4) and gp.shape == (5, 3)
    np.testing.assert_array_equal(go[:, 0], [0, 1, 2, 1, 2])
    np.testing.assert_array_equal(gp[:, 0], [0, 0, 0, 10, 10])
    assert ranks[1]['go'].size == 0


def test_shard_range_properties():
    from spef_amd.shard import shard_range
    for n in (0, 1, 7, 64, 512, 513):
        for w in (1, 2, 3, 8):
            parts = [shard_range(n, r, w) for r in range(w)]
            assert parts[0][0] == 0 and parts[-1][1] == n
            assert all(parts[i][1] == parts[i + 1][0] for i in range(w - 1))
            sizes = [b - a for a, b in parts]
            assert max(sizes) - min(sizes) <= 1
