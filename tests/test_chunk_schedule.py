"""The gathers' chunk schedule as a host model (femasm.hip, k_gather_lin / k_gather_neo: chunk_of):
the resident grid pulls chunks from 8 per-XCD counters, XCD x walking its eighth [x per, (x + 1) per)
of the visiting sequence (lane 0: AHEAD ids from one atomicAdd in the prologue, one atomicInc per
iteration, ids mapped AHEAD iterations early). A workgroup's loop ends at its first empty
descriptor, so the model checks, under random interleavings of the workgroups' counter operations,
that every chunk is gathered exactly once and that no claimed chunk sits behind an empty descriptor.

Also modelled: the tail-stealing variant measured in round 6 (tools/r4/variant.py "steal": past its
eighth a workgroup takes chunks of the other XCDs' eighths; not shipped). Its first
version returned an empty descriptor for the padding positions of the last eighth and then went on to
steal, so a chunk claimed after it was never gathered (found by the deterministic full-size test);
the model fails that version (test_first_steal_version_loses_chunks). The hardware probe
tools/probe/sched_probe.hip runs both schedules on the GPU."""
import random

import pytest

AHEAD = 5  # k_gather_lin: LOOK + 2 chunk ids in flight


class Counters:
    def __init__(self, nchunks, steal=True):
        self.n = nchunks
        self.per = (nchunks + 7) // 8
        self.ctr = [0] * 8
        self.steal = steal

    def len_of(self, x):
        b = x * self.per
        return 0 if b >= self.n else min(self.per, self.n - b)

    def chunk_of(self, xc, j):
        if not self.steal:  # the shipped schedule
            return min(xc * self.per + j, self.n) if j < self.per else self.n
        if j < self.len_of(xc):
            return xc * self.per + j
        for s in range(1, 8):
            v = (xc + s) & 7
            lv = self.len_of(v)
            if self.ctr[v] >= lv:  # the relaxed load
                continue
            r = self.ctr[v]  # atomicInc
            self.ctr[v] += 1
            if r < lv:
                return v * self.per + r
        return self.n


def run(nchunks, nwg, seed, steal=True, cls=Counters):
    rng = random.Random(seed)
    C = cls(nchunks, steal)
    rings = []
    for w in range(nwg):  # the prologue: AHEAD ids from one atomicAdd, mapped in order
        xc = w % 8
        b = C.ctr[xc]
        C.ctr[xc] += AHEAD
        rings.append([C.chunk_of(xc, b + t) for t in range(AHEAD)])
    done = []
    live = list(range(nwg))
    while live:
        w = rng.choice(live)
        ring = rings[w]
        c = ring.pop(0)
        if c >= nchunks:  # the loop ends at the first empty descriptor
            assert all(x >= nchunks for x in ring), f"claimed chunks {ring} behind an empty descriptor"
            live.remove(w)
            continue
        done.append(c)
        xc = w % 8
        j = C.ctr[xc]  # atomicInc on the own counter, mapped AHEAD iterations early
        C.ctr[xc] += 1
        ring.append(C.chunk_of(xc, j))
    return sorted(done)


@pytest.mark.parametrize("steal", [False, True])
@pytest.mark.parametrize("nchunks", [1, 7, 8, 9, 63, 100, 1001, 4097])
@pytest.mark.parametrize("nwg", [8, 16, 64])
def test_every_chunk_once(nchunks, nwg, steal):
    for seed in range(3):
        assert run(nchunks, nwg, seed, steal) == list(range(nchunks))


class FirstSteal(Counters):
    """the first stealing version: no clipping of the last eighths at nchunks"""

    def chunk_of(self, xc, j):
        if j < self.per:
            return min(xc * self.per + j, self.n)
        for s in range(1, 8):
            v = (xc + s) & 7
            if self.ctr[v] >= self.per:
                continue
            r = self.ctr[v]
            self.ctr[v] += 1
            if r < self.per:
                return min(v * self.per + r, self.n)
        return self.n


def test_first_steal_version_loses_chunks():
    bad = 0
    for n in (9, 63, 100, 1001):
        for seed in range(3):
            try:
                bad += run(n, 64, seed, cls=FirstSteal) != list(range(n))
            except AssertionError:
                bad += 1
    assert bad > 0
