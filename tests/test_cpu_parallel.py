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


@pytest.mark.parametrize("ws,gb", [(2, 16), (2, 5), (8, 512), (8, 17)])
def test_gather_and_max_gloo(ws, gb):
    """World sizes 2 and 8 (bench.py --workload c4: 512 images over 8 ranks; 17 over 8 = uneven shards of
    3 and 2): every rank gets the whole batch in order, and the job time is the slowest rank's."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, ws, port, gb, q)) for r in range(ws)]
    for p in procs:
        p.start()
    out = [q.get(timeout=180) for _ in procs]
    for p in procs:
        p.join(60)
        assert p.exitcode == 0
    assert sorted(r for r, _, _ in out) == list(range(ws))
    for rank, vals, t in out:
        assert vals == [float(i) for i in range(gb)]
        assert t == float(ws)


def _noise_worker(rank, ws, port, gb, q):
    """Parity mode: each rank's sampler draws for the full batch in reference order and
    keeps its rows; gathered, the ranks' draws equal one unsharded run's."""
    os.environ.update(RANK=str(rank), WORLD_SIZE=str(ws), LOCAL_RANK=str(rank), MASTER_ADDR="127.0.0.1",
                      MASTER_PORT=str(port))
    from ifd import parallel
    from ifd.sampler import InpaintingSampler
    parallel.init(backend="gloo")
    lo, hi = parallel.shard_range(gb, rank, ws)
    s = InpaintingSampler(None, None, device=torch.device("cpu"), noise_device="cpu", noise_shard=(lo, hi, gb))
    torch.manual_seed(42)
    draws = [s._randn((hi - lo, 3, 8, 8), "cpu") for _ in range(3)]  # img, then per-step noise / known
    full = [parallel.gather_images(d, gb) for d in draws]
    q.put((rank, [f.tolist() for f in full]))
    dist.destroy_process_group()


@pytest.mark.parametrize("gb", [4, 5])
def test_noise_shard_matches_full_batch_gloo(gb):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_noise_worker, args=(r, 2, port, gb, q)) for r in range(2)]
    for p in procs:
        p.start()
    out = [q.get(timeout=120) for _ in procs]
    for p in procs:
        p.join(60)
        assert p.exitcode == 0
    torch.manual_seed(42)
    ref = [torch.randn(gb, 3, 8, 8) for _ in range(3)]
    for rank, full in out:
        for f, r in zip(full, ref):
            assert torch.equal(torch.tensor(f), r)


def test_noise_shard_rejects_mismatched_batch():
    from ifd.sampler import InpaintingSampler
    s = InpaintingSampler(None, None, device=torch.device("cpu"), noise_shard=(2, 4, 8))
    with pytest.raises(ValueError):
        s._randn((3, 3, 8, 8), "cpu")
    with pytest.raises(ValueError):
        InpaintingSampler(None, None, device=torch.device("cpu"), noise_shard=(4, 2, 8))


def test_prepare_gt_mask_broadcasts_and_rejects():
    from ifd.sampler import prepare_gt_mask
    gt = torch.rand(1, 3, 8, 8)
    m = torch.ones(1, 1, 8, 8)
    g2, m2 = prepare_gt_mask(gt, m, 4, 8, 8, "cpu")
    assert g2.shape == (4, 3, 8, 8) and m2.shape == (4, 1, 8, 8) and g2.is_contiguous()
    assert torch.equal(g2[3], gt[0])
    for bad_gt, bad_m in ((torch.rand(2, 3, 8, 8), m), (gt, torch.ones(4, 3, 8, 8)), (gt, torch.ones(4, 1, 4, 4))):
        with pytest.raises(ValueError):
            prepare_gt_mask(bad_gt, bad_m, 4, 8, 8, "cpu")


def test_init_keeps_stdout_clean_gloo(tmp_path):
    """parallel.init under torch.distributed.run (world size 2, gloo): the process group's native connection
    notices go to stderr, so rank 0's stdout holds only what the program prints (bench.py's one JSON line;
    gloo printed "[Gloo] Rank r is connected to ..." there before)."""
    import subprocess
    import sys
    prog = tmp_path / "prog.py"
    prog.write_text("import sys\nsys.path.insert(0, %r)\nfrom ifd import parallel\n"
                    "r, ws, _ = parallel.init(backend='gloo')\nprint('{\"rank\": %%d}' %% r) if r == 0 else None\n"
                    % os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                   "face-inpainting-diffusion-models_amd"))
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    out = subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=2",
                          "--master-addr", "127.0.0.1", f"--master-port={port}", str(prog)],
                         capture_output=True, text=True, timeout=180)
    assert out.returncode == 0, out.stderr[-2000:]
    assert out.stdout.strip() == '{"rank": 0}', out.stdout
