"""Multi-rank path of bench.py / ifd.parallel on CPU with gloo, world_size 2."""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp


def test_shard_range_partitions():
    from ifd.parallel import shard_range
    for gb in (1, 7, 16, 512):
        for ws in (1, 2, 3, 8):
            spans = [shard_range(gb, r, ws) for r in range(ws)]
            assert spans[0][0] == 0 and spans[-1][1] == gb
            assert all(a[1] == b[0] for a, b in zip(spans, spans[1:]))
            assert max(h - l for l, h in spans) - min(h - l for l, h in spans) <= 1


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, ws, port, gb, q):
    os.environ.update(RANK=str(rank), WORLD_SIZE=str(ws), LOCAL_RANK=str(rank), MASTER_ADDR="127.0.0.1",
                      MASTER_PORT=str(port))
    from ifd import parallel
    parallel.init(backend="gloo")
    lo, hi = parallel.shard_range(gb, rank, ws)
    local = torch.arange(lo, hi, dtype=torch.float32).view(-1, 1, 1, 1).expand(-1, 3, 2, 2).contiguous()
    full = parallel.gather_images(local, gb)
    t = parallel.max_over_ranks(float(rank + 1))
    parallel.barrier()
    q.put((rank, full[:, 0, 0, 0].tolist(), t))
    dist.destroy_process_group()


@pytest.mark.parametrize("gb", [16, 5])
def test_gather_and_max_gloo(gb):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, gb, q)) for r in range(2)]
    for p in procs:
        p.start()
    out = [q.get(timeout=120) for _ in procs]
    for p in procs:
        p.join(60)
        assert p.exitcode == 0
    for rank, vals, t in out:
        assert vals == [float(i) for i in range(gb)]
        assert t == 2.0
