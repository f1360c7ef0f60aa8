"""Multi-GPU shard logic on CPU: world_size-2 gloo.

The shards are independent packet ranges, checksummed per rank (here by the oracle,
standing in for each rank's GPU) and never exchanged; the only collective is the
max-over-ranks timing reduction bench.py uses.
"""
import os
import socket

import numpy as np
import pytest
import torch.distributed as dist
import torch.multiprocessing as mp

import _oracle
from _data import ENET_SEED, packed_offsets, ragged_lengths, splitmix64_bytes
import torch
from rusty_enet_amd import crc32_combine
from rusty_enet_amd.shards import max_over_ranks, shard_bounds


@pytest.mark.parametrize("world", [1, 2, 3, 8])
def test_uniform_bounds_partition(world):
    for count in (0, 1, 7, 1 << 20, (1 << 20) + 5):
        b = [shard_bounds(world, r, count=count) for r in range(world)]
        assert b[0][0] == 0 and b[-1][1] == count
        assert all(b[i][1] == b[i + 1][0] for i in range(world - 1))
        assert max(h - l for l, h in b) - min(h - l for l, h in b) <= 1


@pytest.mark.parametrize("world", [2, 4, 8])
def test_ragged_bounds_balance_bytes(world):
    ln = ragged_lengths(ENET_SEED, 100_000)
    b = [shard_bounds(world, r, lengths=ln) for r in range(world)]
    assert b[0][0] == 0 and b[-1][1] == ln.size
    assert all(b[i][1] == b[i + 1][0] for i in range(world - 1))
    total = int(ln.sum())
    for lo, hi in b:
        assert abs(int(ln[lo:hi].sum()) - total / world) <= int(ln.max())


def test_ragged_bounds_edge_cases():
    assert shard_bounds(4, 3, lengths=np.array([], dtype=np.uint32)) == (0, 0)
    one = np.array([1000], dtype=np.uint32)
    b = [shard_bounds(3, r, lengths=one) for r in range(3)]
    assert sum(h - l for l, h in b) == 1
    zeros = np.zeros(10, dtype=np.uint32)  # empty packets: all bytes are 0
    b = [shard_bounds(2, r, lengths=zeros) for r in range(2)]
    assert b[0][0] == 0 and b[-1][1] == 10 and b[0][1] == b[1][0]
    with pytest.raises(ValueError):
        shard_bounds(2, 2, count=4)


def _free_port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _rank_main(rank, world, port, n, result_dir):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        ln = ragged_lengths(ENET_SEED, n)
        off = packed_offsets(ln)
        data = splitmix64_bytes(ENET_SEED + 1, int(ln.sum()))
        lo, hi = shard_bounds(world, rank, lengths=ln)
        # This rank's shard only: its bytes and re-based offsets (what one GPU receives).
        base = int(off[lo]) if hi > lo else 0
        end = int(off[hi - 1] + ln[hi - 1]) if hi > lo else 0
        out = _oracle.crc32_ragged(data[base:end], off[lo:hi] - np.uint64(base), ln[lo:hi])
        np.save(os.path.join(result_dir, f"rank{rank}.npy"), out)
        # Merged digest: the shard's packets fold into the digest of its
        # bytes (packed: the concatenation), then the (crc, bytes) pairs of the ranks
        # fold on rank 0 -- 16 B per rank, host arithmetic (enet_crc32_combine).
        digest = None
        for c, L in zip(out.tolist(), ln[lo:hi].tolist()):
            digest = c if digest is None else crc32_combine(digest, c, L)
        pair = torch.tensor([-1 if digest is None else digest, end - base], dtype=torch.int64)
        pairs = [torch.zeros(2, dtype=torch.int64) for _ in range(world)]
        dist.all_gather(pairs, pair)
        if rank == 0:
            merged = None
            for c, nbytes in (p.tolist() for p in pairs):
                if c >= 0:
                    merged = c if merged is None else crc32_combine(merged, c, nbytes)
            np.save(os.path.join(result_dir, "merged.npy"), np.array([merged], dtype=np.uint64))
        t = max_over_ranks([float(rank + 1), -float(rank)])
        assert t == [float(world), 0.0], t
    finally:
        dist.destroy_process_group()


def test_gloo_world2_shards_cover_batch(tmp_path):
    world, n = 2, 20_000
    mp.start_processes(_rank_main, args=(world, _free_port(), n, str(tmp_path)), nprocs=world,
                       join=True, start_method="spawn")
    got = np.concatenate([np.load(tmp_path / f"rank{r}.npy") for r in range(world)])
    ln = ragged_lengths(ENET_SEED, n)
    data = splitmix64_bytes(ENET_SEED + 1, int(ln.sum()))
    want = _oracle.crc32_ragged(data, packed_offsets(ln), ln)
    assert np.array_equal(got, want)
    assert int(np.load(tmp_path / "merged.npy")[0]) == _oracle.crc32([data])
