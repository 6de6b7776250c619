"""Index model of the one-sided IPC collectives (hccl_amd/csrc/ipc_kernels.hip, geometry from ipc.cc
RunIpcCollective), run on the CPU before any launch. With the kernel's exact loop bounds (vector loop over
[vlo, vhi), element loop from max(vhi*V, lo) to hi), every phase must
  * stay inside each buffer it touches (input, output, a slot of the owner's staging, a result area), and
  * cover each element of each chunk exactly once per phase,
and block b must touch the same piece coordinates in every round of a launch (the per-block barrier relies on it).

An element loop that started at vhi*V wrote one element before a peer's staging for an empty window at the end of a
piece (count 5 on 4 ranks); this model pins the corrected bounds."""
import numpy as np
import pytest

STG_BYTES = 128 << 20  # kIpcStagingBytes (slot area and result area each)
BLOCKS = 128           # kIpcBlocks
AR, RS, RED = 0, 1, 2


def geometry(kind, n, count, es):
    """RunIpcCollective for one launch: (chunks [(start, len)] in input coordinates, piece, block elems, rounds).
    AllReduce: ceil(count/n) rounded to 128 B; ReduceScatter: the blocks; Reduce: the balanced two-shot split."""
    v = 16 // es
    if kind == RS:
        chunks = [(c * count, count) for c in range(n)]
    elif kind == RED:
        base, rem = divmod(count, n)
        chunks = [(c * base + min(c, rem), base + (1 if c < rem else 0)) for c in range(n)]
    else:
        align = 128 // es
        cs = -(-(-(-count // n)) // align) * align
        chunks = [(min(count, c * cs), max(0, min(count, c * cs + cs) - min(count, c * cs))) for c in range(n)]
    widest = max(ln for _, ln in chunks)
    slot_cap = (STG_BYTES // es // n) // v * v
    piece = max(v, min(slot_cap, -(-widest // v) * v))
    block = -(-(-(-piece // BLOCKS)) // v) * v
    rounds = -(-widest // piece)
    return chunks, piece, block, rounds


def piece_len(chunks, c, kp, piece):
    cl = chunks[c][1]
    return 0 if kp >= cl else min(piece, cl - kp)


def touched(lo, hi, v, vec=True):
    vlo = lo // v
    vhi = max(vlo, hi // v) if vec else vlo
    t0 = max(vhi * v, lo)
    return [(vlo * v, vhi * v), (t0, max(t0, hi))]


def check(kind, n, count, es, vec, root=0):
    v = 16 // es
    chunks, piece, block, rounds = geometry(kind, n, count, es)
    total = n * count if kind == RS else count
    out_len = count
    assert n * piece <= STG_BYTES // es
    for me in range(n):
        cover = {ph: np.zeros(total, np.int32) for ph in (0, 1, 2)}
        for k in range(rounds):
            kp = k * piece
            for b in range(BLOCKS):
                for c in range(n):
                    start = chunks[c][0]
                    cvec = vec and start % v == 0  # ChunkVec: element-wise unless the chunk start is aligned
                    plen = piece_len(chunks, c, kp, piece)
                    lo = min(plen, b * block)
                    hi = min(plen, lo + block)
                    assert b * block <= lo or lo == hi          # block b's fixed window, whatever the round
                    for a0, a1 in touched(lo, hi, v, cvec):
                        if a1 <= a0:
                            continue
                        assert lo <= a0 and a1 <= hi
                        g0, g1 = start + kp + a0, start + kp + a1   # input coordinates
                        assert 0 <= g0 and g1 <= total
                        if c != me:
                            assert me * piece + a1 <= n * piece          # owner c's slot me
                            cover[0][g0:g1] += 1
                            if kind == AR or (kind == RED and me == root):
                                assert c * piece + a1 <= n * piece       # my result area, chunk c
                                assert g1 <= out_len
                                cover[2][g0:g1] += 1
                        else:
                            for q in range(n):
                                assert q * piece + a1 <= n * piece       # my slots
                            if kind == RS:
                                assert kp + a1 <= out_len
                            elif kind == RED and me != root:
                                assert me * piece + a1 <= n * piece      # root's result area
                            else:
                                assert g1 <= out_len
                            cover[1][g0:g1] += 1
        for c in range(n):
            start, cl = chunks[c]
            seg = slice(start, start + cl)
            if c == me:
                assert np.all(cover[1][seg] == 1), (me, c)
            else:
                assert np.all(cover[0][seg] == 1), (me, c)
                if kind == AR or (kind == RED and me == root):
                    assert np.all(cover[2][seg] == 1), (me, c)
        if kind != RS:
            assert sum(cl for _, cl in chunks) == count  # the chunks tile the launch exactly


@pytest.mark.parametrize("kind", [AR, RS, RED])
@pytest.mark.parametrize("n", [2, 3, 4, 8, 16])
@pytest.mark.parametrize("es", [1, 2, 4, 8])
@pytest.mark.parametrize("count", [1, 5, 7, 33, 4099, 100003])
def test_ipc_in_bounds_and_exact_cover(kind, n, es, count):
    check(kind, n, count, es, vec=True, root=n - 1)
    check(kind, n, count, es, vec=False, root=0)


@pytest.mark.parametrize("kind,n,count", [(AR, 2, (36 << 20) + 11), (RS, 4, (9 << 20) + 3), (RED, 2, (40 << 20) + 7)])
def test_ipc_multi_round_geometry(kind, n, count):
    """Counts that need several pieces per chunk (fp32): still in bounds, exact cover, fixed block windows."""
    chunks, piece, block, rounds = geometry(kind, n, count, 4)
    assert rounds >= 2
    check(kind, n, count, 4, vec=True, root=1)


def test_old_element_loop_start_is_caught():
    """The pre-fix element loop (from vhi*V) touches an element outside an empty window: the model rejects it."""
    lo = hi = 5
    v = 4
    vhi = hi // v
    bad = (vhi * v, hi)
    assert bad[0] < lo  # would write element 4 for the empty window [5, 5)
    assert touched(lo, hi, v)[1][0] >= lo
