"""Index model of the one-sided IPC AllReduce kernel (hccl_amd/csrc/ipc_kernels.hip), run on the CPU before any
launch: every phase's accesses, with the kernel's exact loop bounds (vector loop over [vlo, vhi), element loop from
max(vhi*V, lo) to hi), must stay inside their buffer and cover each element of the round exactly once.

An element loop that started at vhi*V wrote one element before a peer's staging for an empty range at the end of a
round (count 5, 4 ranks: chunks 2 and 3 are [5, 5)); this model pins the corrected bounds."""
import numpy as np
import pytest

STG_BYTES = 128 << 20  # kIpcStagingBytes (slot area and result area each)
BLOCKS = 128           # kIpcBlocks


def chunk_elems(length, n, v):
    cs = -(-length // n)
    return -(-cs // v) * v


def block_range(length, c, cs, v, b):
    clo = min(length, c * cs)
    chi = min(length, clo + cs)
    bs = -(-(chi - clo) // BLOCKS)
    bs = -(-bs // v) * v
    lo = min(chi, clo + b * bs)
    return lo, min(chi, lo + bs)


def touched(lo, hi, v, vec=True):
    """Element indices CopyRange / the phase-1 loops touch for range [lo, hi) (kernel lines: vlo, vhi, tail)."""
    vlo = lo // v
    vhi = max(vlo, hi // v) if vec else vlo
    tail_start = max(vhi * v, lo)
    return [(vlo * v, vhi * v), (tail_start, max(tail_start, hi))]


def check_round(n, length, es, stg_elems, vec):
    v = 16 // es
    cs = chunk_elems(length, n, v)
    assert n * cs <= stg_elems
    for me in range(n):
        p0 = np.zeros(length, np.int32)   # phase 0: elements of chunk c != me written into owner c's slot me
        p1 = np.zeros(length, np.int32)   # phase 1: elements of chunk me folded
        p2 = np.zeros(length, np.int32)   # phase 2: elements of chunks c != me copied out
        for b in range(BLOCKS):
            for c in range(n):
                lo, hi = block_range(length, c, cs, v, b)
                clo = min(length, c * cs)
                for a0, a1 in touched(lo, hi, v, vec):
                    if a1 <= a0:
                        continue
                    assert lo <= a0 and a1 <= hi, (me, c, b, lo, hi, a0, a1)
                    if c != me:
                        slot0, slot1 = me * cs - clo + a0, me * cs - clo + a1  # stgIn[c] + me*cs - clo + e
                        assert 0 <= slot0 and slot1 <= stg_elems
                        assert a1 <= stg_elems                                 # stgRes[me][e]
                        p0[a0:a1] += 1
                        p2[a0:a1] += 1
                    else:
                        for q in range(n):
                            if q != me:
                                s0, s1 = q * cs - clo + a0, q * cs - clo + a1  # stgIn[me] + q*cs - clo + e
                                assert 0 <= s0 and s1 <= stg_elems
                        p1[a0:a1] += 1
        for c in range(n):
            clo, chi = min(length, c * cs), min(length, c * cs + cs)
            want = 1
            got = (p1 if c == me else p0)[clo:chi]
            assert np.all(got == want), (me, c)
            if c != me:
                assert np.all(p2[clo:chi] == 1)


@pytest.mark.parametrize("n", [2, 3, 4, 5, 8, 16])
@pytest.mark.parametrize("es", [1, 2, 4, 8])
@pytest.mark.parametrize("count", [1, 5, 7, 33, 4096, 4099, 100003, 1 << 20])
@pytest.mark.parametrize("vec", [True, False])
def test_ipc_rounds_in_bounds_and_exact_cover(n, es, count, vec):
    v = 16 // es
    unit = n * v
    round_elems = (STG_BYTES // es) // unit * unit
    base = 0
    while base < count:
        check_round(n, min(round_elems, count - base), es, STG_BYTES // es, vec)
        base += round_elems


@pytest.mark.parametrize("n", [2, 4, 8])
def test_ipc_full_round_fills_staging(n):
    """A full round uses exactly the slot area: n chunks of roundElems / n."""
    es = 4
    v = 16 // es
    unit = n * v
    round_elems = (STG_BYTES // es) // unit * unit
    assert n * chunk_elems(round_elems, n, v) == round_elems <= STG_BYTES // es
