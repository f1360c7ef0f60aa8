"""bench.py's N > 1 line (no GPU): two gloo ranks run bench.main with the GPU work stubbed
out, and rank 0's JSON line must carry the configs[3] main line, the configs[4] shard
timed on every rank (`large_64k`, max over ranks, aggregate value) and one `devices`
entry per rank.  The stubs replace only what needs a GPU; the reduction, the barrier and
the line assembly are bench.py's own."""
import json
import os
import sys

import pytest
import torch.multiprocessing as mp

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)


def _rank(rank: int, world: int, port: int, outdir: str) -> None:
    sys.path.insert(0, REPO)
    import torch

    import bench

    os.environ.update(WORLD_SIZE=str(world), RANK=str(rank), LOCAL_RANK=str(rank), MASTER_ADDR="127.0.0.1",
                      MASTER_PORT=str(port))
    torch.cuda.device_count = lambda: world
    torch.cuda.set_device = lambda d: None
    torch.cuda.synchronize = lambda *a, **k: None
    torch.cuda.empty_cache = lambda: None

    def make_workload(name, rank_, n, dev, length=None):
        L = 65536 if name == "large" else 1200
        return (lambda: None), n * L, n, None, (name,)

    def time_steps(step, steps, barrier, dev):
        barrier()
        for _ in range(steps):
            step()
        barrier()
        # rank r is (r + 1) times slower: the line must report the slowest rank
        return 0.001 * steps * (rank + 1), 0.9 * (rank + 1)

    bench.make_workload = make_workload
    bench.verify_sample = lambda out, spec, limit=20000: None
    bench.open_ceiling = lambda dev: None  # the read-ceiling probe needs a GPU
    bench.time_steps = time_steps
    bench.device_record = lambda dev, r: {"rank": r, "device": dev.index, "pci": f"0000:{0x10 * (r + 1):02x}:00"}
    # Descriptor-level capture: whatever reaches file descriptor 1 (C-level prints such as the
    # gloo transport's connection messages included) is what the driver would read.
    path = os.path.join(outdir, f"stdout{rank}.txt")
    sys.stdout.flush()
    saved = os.dup(1)
    with open(path, "w") as cap:
        os.dup2(cap.fileno(), 1)
        try:
            rc = bench.main(["--gpus", str(world), "--steps", "4", "--warmup", "1", "--cpu-seconds", "0"])
        finally:
            sys.stdout.flush()
            os.dup2(saved, 1)
            os.close(saved)
    with open(path) as f:
        text = f.read()
    with open(os.path.join(outdir, f"rank{rank}.txt"), "w") as f:
        f.write(f"{rc}\n{text}")


def test_multi_gpu_line_shape(tmp_path):
    import socket

    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    world = 2
    mp.start_processes(_rank, args=(world, port, str(tmp_path)), nprocs=world, join=True, start_method="spawn")
    rc0, out0 = (tmp_path / "rank0.txt").read_text().split("\n", 1)
    rc1, out1 = (tmp_path / "rank1.txt").read_text().split("\n", 1)
    assert rc0 == "0" and rc1 == "0" and out1.strip() == ""
    assert len(out0.strip().splitlines()) == 1, out0  # rank 0's stdout: exactly the JSON line
    line = json.loads(out0.strip())
    assert line["n_gpus"] == 2 and line["scaling"] == "weak"
    assert line["config"]["packets_per_gpu"] == 2 << 20  # configs[3]: 16M over 8
    # main line: max over ranks (rank 1 is twice as slow)
    assert line["ms_per_step"] == pytest.approx(2.0)
    assert line["value"] == pytest.approx(2 * (2 << 20) * 1200 / 2e-3 / 2**30, rel=1e-3)
    big = line["large_64k"]
    assert big["n_gpus"] == 2 and big["packets"] == 32768  # configs[4]: 256K over 8
    assert big["ms_per_step"] == pytest.approx(2.0) and big["kernel_ms"] == pytest.approx(1.8)
    # timed twice: right after the warmup (cold) and after SUSTAIN_MS of the point's own launches
    assert big["cold"]["timed_after_launches"] == 1 and big["cold"]["kernel_ms"] > 0
    assert big["timed_after_launches"] >= 1 + 4 and big["timed_after_launches"] * 0.9 >= 60.0
    assert big["value"] == pytest.approx(2 * 32768 * 65536 / 2e-3 / 2**30, rel=1e-3)
    assert big["frac"] == pytest.approx(32768 * 65536 / 1.8e-3 / 1e9 / 8000.0, rel=1e-3)
    assert line["roofline"]["read_ceiling_gbs"] is None and "not built" in line["roofline"]["read_ceiling"]["note"]
    devs = line["devices"]
    assert [d["rank"] for d in devs] == [0, 1] and [d["device"] for d in devs] == [0, 1]
    assert len({d["pci"] for d in devs}) == 2
