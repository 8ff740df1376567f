"""The engine's own halo-exchange posting order, paired across every rank
(host-only; no GPU).

RCCL matches the messages between two ranks purely by the order in which each
posts them inside one ncclGroupStart/End.  lbm_exchange_schedule /
lbm3d_exchange_schedule export the exact list the engines post
(lbm_engine.hip exchange_posts, lbm3d.hip slab_posts -- the RCCL exchange
loops iterate these same lists).  Here every rank's list is generated and
paired the way RCCL pairs it: the k-th send from a to b with the k-th receive
b posts from a.  Each pair must carry the same number of floats, the receive
must fill the ghost side opposite the side the send leaves through, and the
send must go to the sub-domain that actually lies across that side of the
partition (checked from lbm_partition's rectangles, not from the engine's
neighbour table).  Extent-2 dimensions (one peer across two or more sides)
are where order matching can go wrong; 1x1 with the forced exchange sends
every message to itself.  Reference behaviour: the periodic halo slices of
StructuredGridUtils.hpp:805-851.
"""
from __future__ import annotations

import pytest

from lbm_amd import native

DIRS = [(1, 0), (0, 1), (-1, 0), (0, -1), (1, 1), (-1, 1), (-1, -1), (1, -1)]   # E N W S NE NW SW SE
OPP = [2, 3, 0, 1, 6, 7, 4, 5]

GRIDS_2D = [(1, 1), (1, 2), (2, 1), (2, 2), (2, 4), (4, 2), (4, 4), (1, 3), (3, 1), (2, 3), (8, 1), (1, 8)]


def _owner(rects, x, y):
    for r, (x0, y0, w, h) in enumerate(rects):
        if x0 <= x < x0 + w and y0 <= y < y0 + h:
            return r
    raise AssertionError((x, y))


def _pair(scheds, opp=OPP):
    """Pair sends and receives as RCCL does; returns the number of messages."""
    n = 0
    world = len(scheds)
    for a in range(world):
        for b in range(world):
            sends = [x for x in scheds[a] if x[0] == native.XFER_SEND and x[2] == b]
            recvs = [x for x in scheds[b] if x[0] == native.XFER_RECV and x[2] == a]
            assert len(sends) == len(recvs), (a, b, sends, recvs)
            for s, r in zip(sends, recvs):
                assert r[1] == opp[s[1]], (a, b, s, r)   # lands on the ghost side facing the sender
                assert r[3] == s[3], (a, b, s, r)        # same message length
                n += 1
    return n


@pytest.mark.parametrize("mode,width", [(native.HALO_W1, 1), (native.HALO_WG, 2), (native.HALO_WG, 6),
                                        (native.HALO_WG, 10)])
@pytest.mark.parametrize("grid", GRIDS_2D, ids=lambda g: f"{g[0]}x{g[1]}")
@pytest.mark.parametrize("force", [False, True])
def test_2d_schedule_pairs(grid, mode, width, force):
    R, C = grid
    nx, ny = 96 + 5, 80 + 3          # ragged round-robin extents
    parts = R * C
    _, _, rects = native.partition(nx, ny, parts, R, C)
    scheds = [native.exchange_schedule(nx, ny, parts, r, mode, width, R, C, force) for r in range(parts)]
    posted = 0
    for rank, sched in enumerate(scheds):
        x0, y0, w, h = rects[rank]
        # every side appears once as send-or-self, every remote ghost side once as a receive
        assert sorted(d for op, d, _, _ in sched if op != native.XFER_RECV) == list(range(8))
        for op, d, peer, floats in sched:
            dx, dy = DIRS[d]
            if op == native.XFER_RECV:
                dx, dy = -dx, -dy     # the sender sits across ghost side d; its data leaves through OPP(d)
                ex = x0 + (w if DIRS[d][0] > 0 else -1 if DIRS[d][0] < 0 else 0)
                ey = y0 + (h if DIRS[d][1] > 0 else -1 if DIRS[d][1] < 0 else 0)
            else:
                ex = x0 + (w if dx > 0 else -1 if dx < 0 else 0)
                ey = y0 + (h if dy > 0 else -1 if dy < 0 else 0)
            across = _owner(rects, ex % nx, ey % ny)
            assert across == peer, (rank, op, d, peer, across)
            if op == native.XFER_SELF:
                assert peer == rank and not force
                continue
            posted += 1
            side = d if op == native.XFER_SEND else OPP[d]
            edge = (h if side in (0, 2) else w) if side < 4 else 1
            if mode == native.HALO_W1:
                assert floats == (3 if side < 4 else 1) * edge
            else:
                assert floats == 9 * width * (edge if side < 4 else width)
        if force:
            assert all(op != native.XFER_SELF for op, *_ in sched)
    assert _pair(scheds) * 2 == posted


def test_2d_schedule_extent2_repeated_peers():
    """1x2: the E and W neighbours are the same rank, and so are the four
    diagonals' column partners -- several messages to one peer per exchange,
    matched purely by order."""
    scheds = [native.exchange_schedule(64, 32, 2, r, native.HALO_WG, 4, 1, 2) for r in range(2)]
    to_peer = [x for x in scheds[0] if x[0] == native.XFER_SEND and x[2] == 1]
    assert [x[1] for x in to_peer] == [0, 2, 4, 5, 6, 7]
    assert _pair(scheds) == 12


@pytest.mark.parametrize("parts", [1, 2, 3, 4, 5, 8])
@pytest.mark.parametrize("planes", [1, 2, 3])
def test_3d_schedule_pairs(parts, planes):
    nx, ny, nz = 30, 9, 24
    scheds = [native.exchange_schedule3d(nx, ny, nz, parts, r, planes) for r in range(parts)]
    ks = ny * 32
    for rank, sched in enumerate(scheds):
        assert [(op, d) for op, d, _, _ in sched] == [(native.XFER_SEND, 0), (native.XFER_SEND, 1),
                                                     (native.XFER_RECV, 1), (native.XFER_RECV, 0)]
        for op, d, peer, floats in sched:
            assert peer == ((rank + 1) % parts if d == 0 else (rank - 1) % parts)
            assert floats == (5 * ks if planes == 1 else planes * 19 * ks)
    assert _pair(scheds, opp=[1, 0]) == 2 * parts


def test_schedule_rejects_bad_arguments():
    with pytest.raises(native.LbmError):
        native.exchange_schedule(64, 64, 4, 4, native.HALO_WG, 2)      # rank out of range
    with pytest.raises(native.LbmError):
        native.exchange_schedule(64, 64, 4, 0, native.HALO_WG, 0)      # no WG width
    with pytest.raises(native.LbmError):
        native.exchange_schedule(64, 64, 3, 0, native.HALO_W1, 1)      # no rule for 3 parts
    with pytest.raises(native.LbmError):
        native.exchange_schedule3d(8, 8, 4, 5, 0, 1)                   # more slabs than planes
