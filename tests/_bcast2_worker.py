"""Worker of tests/test_gpu_bcast_2rank.py (not collected by pytest): one rank of a 2-GPU torch.distributed.run job.
Rank 0 holds the fp16 blob, rank 1 starts with a different model; spef_bcast_weights must (a) fail cleanly on every
rank, naming rank 1, when rank 1 injects a failure before (SPEF_OPT_TEST_FAIL_BCAST=1) or after (=2) the data
broadcast, leaving rank 1's old model in place, and (b) then deliver rank 0's weights bit for bit (identical logits
on identical frames). Rank 0 prints one JSON line."""
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, 'spacecraft-pose-estimation-framework_amd')]

import numpy as np  # noqa: E402
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402


def main():
    rank, ws, local = int(os.environ['RANK']), int(os.environ['WORLD_SIZE']), int(os.environ['LOCAL_RANK'])
    dev = torch.device(f'cuda:{local}')
    torch.cuda.set_device(dev)
    dist.init_process_group('nccl', rank=rank, world_size=ws, device_id=dev)
    from spef_amd import _lib as L
    from spef_amd import blob as Bl
    from spef_amd.arch import mobilenet_v2
    from spef_amd.engine import Engine
    from spef_amd.shard import RcclComm
    from spef_amd.weights import synthetic_state_dict
    arch = mobilenet_v2('ursonet', 1728, 3)
    eng = Engine(Bl.pack(synthetic_state_dict(arch, seed=1001 if rank == 0 else 7), dtype='fp16'), dev)
    comm = RcclComm(dev, timeout_ms=30_000)
    fr = torch.from_numpy(np.random.Generator(np.random.PCG64(3)).integers(0, 256, (2, 96, 128, 3),
                                                                            dtype=np.uint8)).to(dev)
    o_old, _ = eng.forward(fr)
    res = {}
    for mode in (1, 2):
        eng.set_option(L.OPT_TEST_FAIL_BCAST, mode if rank == 1 else 0)
        try:
            eng.bcast_weights(comm, 0)
            res[f'fail{mode}'] = [0, '']
        except L.SpefError as e:
            res[f'fail{mode}'] = [int(e.code), str(e)]
        o, _ = eng.forward(fr)
        res[f'fail{mode}_model_kept'] = bool(torch.equal(o, o_old))
    eng.set_option(L.OPT_TEST_FAIL_BCAST, 0)
    eng.bcast_weights(comm, 0)
    o, p = eng.forward(fr)
    logits = [torch.zeros_like(o) for _ in range(ws)]
    dist.all_gather(logits, o.contiguous())
    every = [None] * ws
    dist.all_gather_object(every, res)
    if rank == 0:
        print(json.dumps({'ranks': every, 'identical_after_bcast': all(torch.equal(logits[0], t) for t in logits[1:]),
                          'rank1_changed': not torch.equal(logits[1], o_old) if ws > 1 else None}), flush=True)
    comm.close()
    eng.close()
    dist.barrier()
    dist.destroy_process_group()


if __name__ == '__main__':
    main()
