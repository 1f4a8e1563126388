"""StreamPipeline (batches alternating over HIP streams, spef_amd/pipeline.py): every batch's pose equals the
single-stream engine's, bit for bit, whatever the interleaving."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


def test_pipeline_matches_single_stream():
    from oracle import decode_ref as D
    from spef_amd import blob as Bl
    from spef_amd.arch import mobilenet_v2
    from spef_amd.engine import Engine
    from spef_amd.pipeline import StreamPipeline
    from spef_amd.weights import synthetic_state_dict

    blob = Bl.pack(synthetic_state_dict(mobilenet_v2('ursonet', 1728, 3), seed=7), dtype='fp16')
    h, _ = D.orientation_histogram(12, False)
    rng = np.random.Generator(np.random.PCG64(3))
    batches = [torch.from_numpy(rng.integers(0, 256, (4, 128, 160, 3), dtype=np.uint8)).cuda() for _ in range(7)]
    ref = Engine(blob, 'cuda:0')
    ref.set_decode_tables(h, None)
    want = []
    for x in batches:
        o, p = ref.forward(x)
        d = ref.decode(1, 0, o, p)
        want.append((d['ori'].cpu().numpy(), d['pos'].cpu().numpy(), d['ori_soft'].cpu().numpy()))
    ref.close()
    pipe = StreamPipeline(blob, 'cuda:0', depth=3, ori_bins=h)
    got = [pipe.submit(x) for x in batches]
    pipe.synchronize()
    for (q, t, s), d in zip(want, got):
        assert np.array_equal(q, d['ori'].cpu().numpy())
        assert np.array_equal(t, d['pos'].cpu().numpy())
        assert np.array_equal(s, d['ori_soft'].cpu().numpy())
        assert not d['status'].any().item()
    pipe.close()


def test_pipeline_graph_replay_matches_single_stream():
    """use_graphs(): each (stream, batch) pair's forward + decode recorded once as a HIP graph and replayed. Two rounds
    over the same 3 batches on 3 streams (recorded in round 1, replayed in round 2) equal the single-stream engine's
    outputs bit for bit, and round 2 replays rather than records (same output storage as round 1)."""
    from oracle import decode_ref as D
    from spef_amd import blob as Bl
    from spef_amd.arch import mobilenet_v2
    from spef_amd.engine import Engine
    from spef_amd.pipeline import StreamPipeline
    from spef_amd.weights import synthetic_state_dict

    blob = Bl.pack(synthetic_state_dict(mobilenet_v2('ursonet', 1728, 3), seed=7), dtype='fp16')
    h, _ = D.orientation_histogram(12, False)
    rng = np.random.Generator(np.random.PCG64(5))
    batches = [torch.from_numpy(rng.integers(0, 256, (4, 128, 160, 3), dtype=np.uint8)).cuda() for _ in range(3)]
    ref = Engine(blob, 'cuda:0')
    ref.set_decode_tables(h, None)
    want = []
    for x in batches:
        o, p = ref.forward(x)
        d = ref.decode(1, 0, o, p)
        want.append((d['ori'].cpu().numpy(), d['pos'].cpu().numpy(), d['ori_soft'].cpu().numpy()))
    ref.close()
    pipe = StreamPipeline(blob, 'cuda:0', depth=3, ori_bins=h)
    pipe.use_graphs()
    first = [pipe.submit(x) for x in batches]
    pipe.synchronize()
    for d in first:   # clobber round 1's outputs: round 2 must rewrite them
        d['ori'].fill_(7.0)
        d['pos'].fill_(7.0)
    torch.cuda.synchronize()
    second = [pipe.submit(x) for x in batches]
    pipe.synchronize()
    assert len(pipe._graphs) == 3
    for (q, t, s), d1, d2 in zip(want, first, second):
        assert d1['ori'].data_ptr() == d2['ori'].data_ptr()
        assert np.array_equal(q, d2['ori'].cpu().numpy())
        assert np.array_equal(t, d2['pos'].cpu().numpy())
        assert np.array_equal(s, d2['ori_soft'].cpu().numpy())
        assert not d2['status'].any().item()
    pipe.close()


def test_pipeline_graphs_dropped_when_buffers_move():
    """a recorded graph holds fixed device addresses (workspace, output buffers), so a batch-size
    change on a stream (new output buffers, a larger workspace) must drop that stream's graphs. Record at B = 4, submit
    B = 8 on the same stream (workspace reallocated), then B = 4 again: every output equals the eager engine's."""
    from oracle import decode_ref as D
    from spef_amd import blob as Bl
    from spef_amd.arch import mobilenet_v2
    from spef_amd.engine import Engine
    from spef_amd.pipeline import StreamPipeline
    from spef_amd.weights import synthetic_state_dict

    blob = Bl.pack(synthetic_state_dict(mobilenet_v2('ursonet', 1728, 3), seed=7), dtype='fp16')
    h, _ = D.orientation_histogram(12, False)
    rng = np.random.Generator(np.random.PCG64(9))
    x4 = torch.from_numpy(rng.integers(0, 256, (4, 128, 160, 3), dtype=np.uint8)).cuda()
    x8 = torch.from_numpy(rng.integers(0, 256, (8, 128, 160, 3), dtype=np.uint8)).cuda()
    ref = Engine(blob, 'cuda:0')
    ref.set_decode_tables(h, None)
    want = {}
    for k, x in (('4', x4), ('8', x8)):
        o, p = ref.forward(x)
        want[k] = ref.decode(1, 0, o, p)['ori'].cpu().numpy()
    ref.close()
    pipe = StreamPipeline(blob, 'cuda:0', depth=1, ori_bins=h)
    pipe.use_graphs()
    try:
        for k, x in (('4', x4), ('8', x8), ('4', x4), ('4', x4)):
            d = pipe.submit(x)
            pipe.synchronize()
            assert np.array_equal(d['ori'].cpu().numpy(), want[k]), k
            assert not d['status'].any().item()
        assert len(pipe._graphs) == 1   # only the graph recorded against the current buffers survives
    finally:
        pipe.close()
