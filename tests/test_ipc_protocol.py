"""Model check of the IPC kernel's cross-rank protocol (hccl_amd/csrc/ipc_kernel_body.h k_ipc_collective, ipc.cc).

Ranks are streams of launches; a launch is `blocks` workgroups, each running the kernel's per-round steps. One step
runs at a time, and a random scheduler picks which, so many interleavings of blocks and ranks are tried:
  * phase 0: block b of rank i stores its window of the round's piece into every owner's slot i;
  * barrier e: stores epoch e into flag[c][b][i] of every rank c, then waits until flag[i][b][c] >= e for every c;
  * phase 1: the fold reads every slot of its window (begin ... end, other steps may run in between) and, for the
    two-shot AllReduce, stores the result into every peer's result area;
  * second barrier and phase 2 (two-barrier kinds only): reads the result area.
The slot area is stgIn for the two-barrier kinds and, for the single-barrier kinds (ReduceScatter, one-shot
AllReduce / Reduce), alternate area (e & 1) of the round's barrier epoch e. A rank starts its next launch only when
every block of the current one has finished (stream order).

Checked on every element: a fold or phase-2 read sees exactly the current round's data from the right rank, and no
store lands on an element while a read of it is in progress. The same model with the alternation switched off
(single-barrier kinds on stgIn) must fail: that is the race the second barrier used to prevent.
"""
import random

import pytest

SINGLE, DOUBLE = "single", "double"


def _launches(rng, count):
    """Launch descriptors: kind, rounds, block count and piece (elements), varying from launch to launch."""
    out = []
    for _ in range(count):
        kind = rng.choice((SINGLE, SINGLE, DOUBLE))
        blocks = rng.choice((1, 2, 3, 4))
        piece = rng.choice((4, 5, 8, 12))
        out.append((kind, rng.choice((1, 2, 3)), blocks, piece))
    return out


class Violation(AssertionError):
    pass


M32 = 1 << 32


def _run(n, launches, seed, alternate=True, max_steps=200000, epoch_base=0, wrap_safe=True):
    """epoch_base: value of the device epoch counter (and of every flag) before the first launch; the kernel's 32-bit
    epochs are taken modulo 2^32, so a base near 2^32 runs the barriers across the wrap. wrap_safe: the kernel's
    `(int32_t)(flag - epoch) < 0` wait; False models a plain unsigned `flag < epoch`."""
    rng = random.Random(seed)
    cap = 16  # elements per slot in every area
    areas = ("in", "res", "alt0", "alt1")
    # tag[owner][area][slot][elem] = (global round id, writer rank); readers[...] = reads in progress
    tag = {(o, a, q, x): None for o in range(n) for a in areas for q in range(n) for x in range(cap)}
    readers = {k: 0 for k in tag}
    flags = {}  # (owner, block, sender) -> last stored epoch, modulo 2^32

    def behind(flag, ep):
        if wrap_safe:
            d = (flag - ep) % M32
            return d >= (1 << 31)  # (int32_t)(flag - ep) < 0
        return flag < ep

    def store(owner, area, slot, lo, hi, val):
        for x in range(lo, hi):
            k = (owner, area, slot, x)
            if readers[k]:
                raise Violation(f"store to {k} during a read")
            tag[k] = val

    def begin_read(owner, area, slot, lo, hi, want):
        for x in range(lo, hi):
            k = (owner, area, slot, x)
            if tag[k] != want:
                raise Violation(f"read of {k} saw {tag[k]}, want {want}")
            readers[k] += 1

    def end_read(owner, area, slot, lo, hi):
        for x in range(lo, hi):
            readers[(owner, area, slot, x)] -= 1

    def program(me, lid, launch, b, epoch0, round0):
        """The step list of block b of rank `me` in launch `lid` (mirrors k_ipc_collective)."""
        kind, rounds, blocks, piece = launch
        be = -(-piece // blocks)
        lo, hi = min(piece, b * be), min(piece, (b + 1) * be)
        steps, e = [], epoch0
        for k in range(rounds):
            g = round0 + k
            area = (f"alt{(e + 1) & 1}" if alternate else "in") if kind == SINGLE else "in"
            steps += [("store", c, area, me, lo, hi, (g, me)) for c in range(n) if c != me]
            e += 1
            steps.append(("wait", e))
            steps += [("begin", me, area, q, lo, hi, (g, q)) for q in range(n) if q != me]
            if kind == DOUBLE:  # two-shot: push the result to every peer's result area
                steps += [("store", p, "res", me, lo, hi, (g, "res", me)) for p in range(n) if p != me]
            steps += [("end", me, area, q, lo, hi) for q in range(n) if q != me]
            if kind == DOUBLE:
                e += 1
                steps.append(("wait", e))
                steps += [("begin", me, "res", c, lo, hi, (g, "res", c)) for c in range(n) if c != me]
                steps += [("end", me, "res", c, lo, hi) for c in range(n) if c != me]
        return steps

    # epoch base and global round id of each launch: equal on every rank, as ipc.cc computes them
    bases, e, g = [], 0, 0
    for kind, rounds, blocks, piece in launches:
        bases.append((e, g))
        e += rounds * (1 if kind == SINGLE else 2)
        g += rounds
    cur = [0] * n  # launch index per rank
    progs = {}
    pc = {}

    def start(me):
        lid = cur[me]
        if lid < len(launches):
            for b in range(launches[lid][2]):
                progs[(me, b)] = program(me, lid, launches[lid], b, *bases[lid])
                pc[(me, b)] = 0
        return lid < len(launches)

    def advance(me):
        """Start rank me's next launch if every block of its current one has finished (stream order)."""
        mine = [k for k in progs if k[0] == me]
        if cur[me] >= len(launches) or not all(pc[k] >= len(progs[k]) for k in mine):
            return False
        for k in mine:
            del progs[k]
            del pc[k]
        cur[me] += 1
        start(me)
        return True

    signalled = set()
    for me in range(n):
        start(me)
    for _ in range(max_steps):
        if all(cur[me] >= len(launches) for me in range(n)):
            return
        # a rank whose launch is finished starts the next one at a random later step
        if any(advance(me) for me in range(n) if rng.random() < 0.3):
            continue
        live = [k for k in progs if pc[k] < len(progs[k])]
        rng.shuffle(live)
        progressed = False
        for me, b in live:
            step = progs[(me, b)][pc[(me, b)]]
            if step[0] == "wait":
                ep = step[1]
                if (me, b, ep) not in signalled:  # the barrier's release store to every rank's flag
                    signalled.add((me, b, ep))
                    for c in range(n):
                        flags[(c, b, me)] = (epoch_base + ep) % M32  # a block signals its epochs in order
                    progressed = True
                    break
                if any(behind(flags.get((me, b, c), epoch_base % M32), (epoch_base + ep) % M32) for c in range(n)):
                    continue  # still waiting: try another block
            elif step[0] == "store":
                store(*step[1:])
            elif step[0] == "begin":
                begin_read(*step[1:])
            else:
                end_read(*step[1:])
            pc[(me, b)] += 1
            progressed = True
            break
        if not progressed and not any([advance(me) for me in range(n)]):
            raise Violation("deadlock")
    raise Violation("step limit")


@pytest.mark.parametrize("n", [2, 3, 4])
def test_protocol_is_race_free(n):
    for seed in range(60):
        rng = random.Random(1000 * n + seed)
        _run(n, _launches(rng, 6), seed)


def test_single_barrier_without_alternation_races():
    """Negative control: the single-barrier kinds folding from stgIn with no second barrier must be caught."""
    found = 0
    for seed in range(200):
        rng = random.Random(seed)
        try:
            _run(3, [(SINGLE, 3, 2, 8)] + _launches(rng, 3), seed, alternate=False)
        except Violation:
            found += 1
    assert found > 0


@pytest.mark.parametrize("n", [2, 3])
def test_protocol_is_race_free_across_epoch_wrap(n):
    """The epoch counter never resets: 2^31 two-shot calls wrap it. Starting just below 2^32, every barrier of the
    launches below crosses the wrap; the wrap-safe compare keeps the protocol exact."""
    for seed in range(40):
        rng = random.Random(7000 * n + seed)
        _run(n, _launches(rng, 6), seed, epoch_base=M32 - 5)


def test_unsigned_compare_breaks_at_the_wrap():
    """Negative control: with `flag < epoch` a barrier after the wrap opens without waiting."""
    found = 0
    for seed in range(100):
        rng = random.Random(seed)
        try:
            _run(3, [(SINGLE, 3, 2, 8), (DOUBLE, 3, 2, 8)] + _launches(rng, 2), seed, epoch_base=M32 - 3,
                 wrap_safe=False)
        except Violation:
            found += 1
    assert found > 0
