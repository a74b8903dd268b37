"""Item-block rotation between ranks, checked on CPU with gloo.

mfhip's rank mode (csrc/mfhip.cpp ring_shift) moves item blocks with RCCL send/recv after every
superstep: rank g owns user blocks g*c .. g*c+c-1 (n = c * world), sends item block
(g*c + s - 1) mod n to rank g-1 and receives ((g+1)*c + s - 1) mod n from rank g+1 -- the
reference's nextRatingBlock (DSGDforMF.scala:611-619).  RCCL cannot run two ranks on the one
GPU of the test box, so this test runs the same protocol over gloo send/recv (a block = a
tensor carrying its id and an update log) with world sizes 2, 4 and 8 (n = 16, c = 2).  The
blocks each rank sends and receives and its peers come from the LIBRARY's own ring step
(mf_debug_ring_schedule, the function ring_shift calls; no GPU needed), so a change to the C++
indices breaks this test.  It checks that

  * at superstep s every rank holds exactly the item blocks (p + s - 1) mod n of its user
    blocks p (the rating blocks DSGDforMF.scala:429-439 matches),
  * over n supersteps every rating block (p, q) is visited exactly once,
  * every item block sees its user blocks in the same order as a single-process run.
"""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def ring_step(rank, world, n, s):
    """The library's ring step after superstep s: (out_blk, in_blk, dst, src)."""
    import ctypes as C
    from mfhip import _lib as L
    vals = [C.c_int32(0) for _ in range(4)]
    L.check(L.lib().mf_debug_ring_schedule(rank, world, n, s, *[C.byref(v) for v in vals]))
    return tuple(v.value for v in vals)


def _rank_main(rank, world, n, epochs, port, out):
    import sys
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                    "large-scale-recommendation_amd"))
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    c = n // world
    # item block q starts on the rank owning user block q (reset_item_loc: q / c)
    held = {q: torch.tensor([q] + [-1] * (n * epochs), dtype=torch.int64) for q in range(rank * c, rank * c + c)}
    fill = {q: 0 for q in held}
    visited = []
    for s in range(1, n * epochs + 1):
        for j in range(c):
            p = rank * c + j
            q = (p + s - 1) % n
            assert q in held, (rank, s, q, sorted(held))
            visited.append((p, q))
            fill[q] += 1
            held[q][fill[q]] = p  # "update" the item block with user block p
        out_blk, in_blk, dst, src = ring_step(rank, world, n, s)
        buf = torch.empty_like(held[out_blk])
        send_req = dist.isend(held.pop(out_blk), dst=dst)
        dist.recv(buf, src=src)
        send_req.wait()
        assert int(buf[0]) == in_blk
        fill.pop(out_blk)
        held[in_blk] = buf
        fill[in_blk] = int((buf[1:] >= 0).sum())
    blocks = [None] * world
    dist.all_gather_object(blocks, ({q: t.tolist() for q, t in held.items()}, visited))
    if rank == 0:
        out.put(blocks)
    dist.barrier()
    dist.destroy_process_group()


def _single_process(n, epochs):
    logs = {q: [] for q in range(n)}
    for s in range(1, n * epochs + 1):
        for p in range(n):
            logs[(p + s - 1) % n].append(p)
    return logs


def test_library_ring_step_is_next_rating_block():
    """mf_debug_ring_schedule against nextRatingBlock (DSGDforMF.scala:611-619) restated: after
    superstep s rank g's first rating block (g*c, (g*c+s-1) mod n) becomes (g*c-1, same q), owned by
    rank g-1; its item block comes from rank g+1."""
    for world, n in [(1, 3), (2, 4), (4, 8), (8, 16), (8, 8)]:
        c = n // world
        for s in range(1, 2 * n + 1):
            for g in range(world):
                out_blk, in_blk, dst, src = ring_step(g, world, n, s)
                assert out_blk == (g * c + s - 1) % n and dst == (g - 1) % world
                assert src == (g + 1) % world and in_blk == ring_step(src, world, n, s)[0]


@pytest.mark.parametrize("world,n", [(2, 4), (2, 8), (4, 8), (8, 16)])
def test_item_block_rotation_over_gloo(world, n):
    epochs = 2
    ctx = mp.get_context("spawn")
    out = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_rank_main, args=(r, world, n, epochs, port, out)) for r in range(world)]
    for p in procs:
        p.start()
    blocks = out.get(timeout=120)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    visited = [v for _, vis in blocks for v in vis]
    assert sorted(visited) == sorted((p, q) for p in range(n) for q in range(n) for _ in range(epochs))
    held = {}
    for h, _ in blocks:
        held.update(h)
    assert sorted(held) == list(range(n))
    ref = _single_process(n, epochs)
    for q, log in held.items():
        assert log[0] == q
        assert [x for x in log[1:] if x >= 0] == ref[q]
