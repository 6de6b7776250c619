"""Index model of the one-sided IPC collectives (hccl_amd/csrc/ipc_kernel_body.h, geometry from ipc.cc
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
AR1, RED1, ARMC = 3, 4, 5  # one-shot AllReduce, one-shot Reduce, MeshChunk AllReduce (order O6, unaligned ceil)
ARBAL = 6  # AIV large-core two-shot AllReduce: group * n balanced slices, rank c owning [c*group, (c+1)*group)


RSV = 7  # ReduceScatterV: kIpcGeomV, chunk c = (displs[c], counts[c]), any alignment, order O1


def geometry(kind, n, count, es, group=1, vblocks=None):
    """RunIpcCollective for one launch: (chunks [(start, len)] in input coordinates, piece, block elems, rounds).
    AllReduce: ceil(count/n) rounded to 128 B; ReduceScatter: the blocks; Reduce: the balanced two-shot split;
    one-shot kinds: every chunk is the whole range; MeshChunk AllReduce: ceil(count/n) without alignment."""
    v = 16 // es
    if kind == RSV:
        chunks = list(vblocks)
    elif kind in (AR1, RED1):
        chunks = [(0, count) for _ in range(n)]
    elif kind == ARMC:
        cs = -(-count // n)
        chunks = [(min(count, c * cs), max(0, min(count, c * cs + cs) - min(count, c * cs))) for c in range(n)]
    elif kind == RS:
        chunks = [(c * count, count) for c in range(n)]
    elif kind in (RED, ARBAL):
        # kIpcGeomBalanced: group * n slices, chunk c = slices [c*group, (c+1)*group) (Reduce two-shot: group 1)
        g = group if kind == ARBAL else 1
        base, rem = divmod(count, g * n)
        chunks = [(c * g * base + min(c * g, rem), g * base + max(0, min(g, rem - c * g))) for c in range(n)]
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


def shares(plen, b, block, tile, blocks=BLOCKS):
    """ipc_kernel_body.h ForBlockShare: block b's ranges of piece coordinates [0, plen) -- one window of `block`
    elements (tile == 0, BlockWindow), or tiles of `tile` elements at b, b + B, ... (B = blocks)."""
    if tile == 0:
        lo = min(plen, b * block)
        return [(lo, min(plen, lo + block))]
    return [(lo, min(plen, lo + tile)) for lo in range(b * tile, plen, blocks * tile)]


def piece_len(chunks, c, kp, piece):
    cl = chunks[c][1]
    return 0 if kp >= cl else min(piece, cl - kp)


def touched(lo, hi, v, vec=True):
    vlo = lo // v
    vhi = max(vlo, hi // v) if vec else vlo
    t0 = max(vhi * v, lo)
    return [(vlo * v, vhi * v), (t0, max(t0, hi))]


def sub_starts(length, n, es, rs4k):
    """Sub-slice starts of a chunk for order O6 (ipc_kernel_body.h SubStart), plus the end."""
    parts = n - 1
    if rs4k and parts >= 2:
        al = length * es // parts // 4096 * 4096 // es
        if al:
            return [j * al for j in range(parts)] + [length]
    base, big = divmod(length, parts)
    return [j * base + min(j, big) for j in range(parts)] + [length]


def fold_touched(lo, hi, v, vec):
    """FoldSeg's accesses for [lo, hi): scalar head up to a vector boundary, the vector body, the scalar tail."""
    vb, ve = -(-lo // v), hi // v
    if not vec or vb >= ve:
        return [(lo, hi)]
    return [(lo, vb * v), (vb * v, ve * v), (ve * v, hi)]


def fold_segments(kind, n, es, chunk_len, kp, lo, hi, o6):
    """FoldRange: the window, or its pieces per O6 sub-slice (piece coordinates)."""
    if not o6 or n < 2:
        return [(lo, hi)]
    st = sub_starts(chunk_len, n, es, kind == RS)
    out = []
    for j in range(n - 1):
        a0 = max(lo, st[j] - kp if st[j] > kp else 0)
        a1 = min(hi, st[j + 1] - kp if st[j + 1] > kp else 0)
        if a0 < a1:
            out.append((a0, a1))
    return out


def check_general(kind, n, count, es, vec, root=0, o6=False, vblocks=None, tile=0):
    """The generalised kernel: one-shot kinds push the whole piece (Reduce: to the root only) and fold it without a
    phase 2; O6 folds a window per sub-slice with scalar head and tail around the vector body."""
    v = 16 // es
    chunks, piece, block, rounds = geometry(kind, n, count, es, vblocks=vblocks)
    total = n * count if kind == RS else count
    if kind == RSV:
        total = max(st + ln for st, ln in chunks)
    for me in range(n):
        cover1 = np.zeros(total, np.int32)
        pushed = np.zeros((n, total), np.int32)  # pushed[c]: elements delivered to owner c by me
        for k in range(rounds):
            kp = k * piece
            for b in range(BLOCKS):
                for c in range(n):
                    start, cl = chunks[c]
                    plen = 0 if kp >= cl else min(piece, cl - kp)
                    cvec = vec and start % v == 0
                    for lo, hi in shares(plen, b, block, tile):
                        if c != me and not (kind == RED1 and c != root):
                            for a0, a1 in touched(lo, hi, v, cvec):
                                if a1 > a0:
                                    assert me * piece + a1 <= n * piece
                                    pushed[c][start + kp + a0:start + kp + a1] += 1
                        if c == me and not (kind == RED1 and me != root):
                            for s0, s1 in fold_segments(kind, n, es, cl, kp, lo, hi, o6):
                                for a0, a1 in fold_touched(s0, s1, v, cvec):
                                    if a1 <= a0:
                                        continue
                                    assert lo <= a0 and a1 <= hi
                                    for q in range(n):
                                        assert q * piece + a1 <= n * piece
                                    g0, g1 = start + kp + a0, start + kp + a1
                                    assert 0 <= g0 and g1 <= total
                                    cover1[g0:g1] += 1
        for c in range(n):
            start, cl = chunks[c]
            seg = slice(start, start + cl)
            if c == me:
                if not (kind == RED1 and me != root):
                    assert np.all(cover1[seg] == 1), (kind, me, c)
            elif not (kind == RED1 and c != root):
                assert np.all(pushed[c][seg] == 1), (kind, me, c)


@pytest.mark.parametrize("kind", [AR1, RED1])
@pytest.mark.parametrize("n", [2, 3, 8])
@pytest.mark.parametrize("es", [1, 2, 4, 8])
@pytest.mark.parametrize("count", [1, 5, 33, 4099, 100003])
def test_ipc_one_shot_in_bounds_and_exact_cover(kind, n, es, count):
    check_general(kind, n, count, es, vec=True, root=n - 1)
    check_general(kind, n, count, es, vec=False, root=0)


@pytest.mark.parametrize("kind", [ARMC, RS])
@pytest.mark.parametrize("n", [2, 3, 4, 8])
@pytest.mark.parametrize("es", [1, 2, 4, 8])
@pytest.mark.parametrize("count", [1, 7, 33, 4099, 70001, 300007])
def test_ipc_o6_sub_slices_in_bounds_and_exact_cover(kind, n, es, count):
    """Order O6 folds a block's window per sub-slice; sub-slice edges fall anywhere (scalar head/tail)."""
    check_general(kind, n, count, es, vec=True, o6=True)
    check_general(kind, n, count, es, vec=False, o6=True)


def check_allgather(n, count, es, vec, blocks):
    """kIpcAllGather: the one-shot geometry (every rank pushes its whole piece to every peer's slot `me`), then each
    rank copies slot q (its own piece from its input) to output block q at q * count. Every output element is written
    exactly once per rank, inside [0, n * count), and every slot access stays inside the owner's n slots."""
    v = 16 // es
    slot_cap = (STG_BYTES // es // n) // v * v
    piece = max(v, min(slot_cap, -(-count // v) * v))
    block = -(-(-(-piece // blocks)) // v) * v
    rounds = -(-count // piece)
    for me in range(n):
        out_cover = np.zeros(n * count, np.int32)
        pushed = np.zeros(count, np.int32)
        for k in range(rounds):
            kp = k * piece
            plen = 0 if kp >= count else min(piece, count - kp)
            for b in range(blocks):
                lo = min(plen, b * block)
                hi = min(plen, lo + block)
                for a0, a1 in touched(lo, hi, v, vec):
                    if a1 > a0:
                        assert me * piece + a1 <= n * piece
                        pushed[kp + a0:kp + a1] += 1  # once per peer: counted for one of them
                for q in range(n):
                    for a0, a1 in touched(lo, hi, v, vec and (q * count) % v == 0):
                        if a1 <= a0:
                            continue
                        assert q * piece + a1 <= n * piece
                        g0, g1 = q * count + kp + a0, q * count + kp + a1
                        assert 0 <= g0 and g1 <= n * count
                        out_cover[g0:g1] += 1
        assert np.all(pushed == 1), me
        assert np.all(out_cover == 1), me


def default_blocks(nbytes):
    """ipc.cc DefaultIpcBlocks: workgroups per launch by the call's bytes."""
    for limit, b in ((64 << 10, 4), (512 << 10, 16), (2 << 20, 32), (32 << 20, 64), (64 << 20, 128)):
        if nbytes <= limit:
            return b
    return 256


@pytest.mark.parametrize("n", [2, 3, 8])
@pytest.mark.parametrize("es", [1, 2, 4, 8])
@pytest.mark.parametrize("count", [1, 5, 33, 4099, 100003])
def test_ipc_allgather_in_bounds_and_exact_cover(n, es, count):
    for blocks in sorted({default_blocks(n * count * es), 1, 256}):
        check_allgather(n, count, es, vec=True, blocks=blocks)
        check_allgather(n, count, es, vec=False, blocks=blocks)


def test_ipc_allgather_multi_round():
    n, count = 2, (36 << 20) + 11  # fp32: 3 rounds of 16 Mi elements
    check_allgather(n, count, 4, vec=True, blocks=default_blocks(n * count * 4))


def check(kind, n, count, es, vec, root=0, group=1, tile=0):
    v = 16 // es
    chunks, piece, block, rounds = geometry(kind, n, count, es, group)
    two_shot = kind in (AR, ARBAL)
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
                    for lo, hi, a0, a1 in ((lo, hi, a0, a1) for lo, hi in shares(plen, b, block, tile)
                                           for a0, a1 in touched(lo, hi, v, cvec)):
                        # block b's fixed coordinates, whatever the round
                        assert (b * block <= lo or lo == hi) if tile == 0 else (lo // tile) % BLOCKS == b
                        if a1 <= a0:
                            continue
                        assert lo <= a0 and a1 <= hi
                        g0, g1 = start + kp + a0, start + kp + a1   # input coordinates
                        assert 0 <= g0 and g1 <= total
                        if c != me:
                            assert me * piece + a1 <= n * piece          # owner c's slot me
                            cover[0][g0:g1] += 1
                            if two_shot or (kind == RED and me == root):
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
                if two_shot or (kind == RED and me == root):
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


@pytest.mark.parametrize("n,group", [(2, 22), (4, 8), (8, 4), (8, 1), (16, 1)])
@pytest.mark.parametrize("es", [1, 2, 4, 8])
@pytest.mark.parametrize("count", [1, 5, 33, 4099, 100003, 1 << 20])
def test_ipc_aiv_balanced_groups_in_bounds_and_exact_cover(n, group, es, count):
    """The AIV large-core two-shot's chunks (group * n balanced slices per loop, group = (blocks - n) / n for the
    default 48 vector cores: 22 at n = 2, 8 at n = 4, 4 at n = 8): chunk starts fall anywhere."""
    check(ARBAL, n, count, es, vec=True, group=group)
    check(ARBAL, n, count, es, vec=False, group=group)


def test_old_element_loop_start_is_caught():
    """The pre-fix element loop (from vhi*V) touches an element outside an empty window: the model rejects it."""
    lo = hi = 5
    v = 4
    vhi = hi // v
    bad = (vhi * v, hi)
    assert bad[0] < lo  # would write element 4 for the empty window [5, 5)
    assert touched(lo, hi, v)[1][0] >= lo


@pytest.mark.parametrize("layout", ["ragged", "gapped", "overlap", "empty", "unaligned"])
@pytest.mark.parametrize("n", [2, 3, 8])
@pytest.mark.parametrize("es", [1, 2, 4, 8])
def test_ipc_reduce_scatter_v_in_bounds_and_exact_cover(layout, n, es):
    """kIpcGeomV (HcclReduceScatterV on the one-sided kernel): blocks of any size at any displacement, overlapping
    or empty; every block pushed to its owner once and folded by it once, inside every buffer."""
    if layout == "gapped":
        blocks = [(q * 9001 + 3, 7001) for q in range(n)]
    elif layout == "overlap":
        blocks = [(q * 100, 30007) for q in range(n)]
    elif layout == "empty":
        blocks = [(q * 5000, 0 if q == 1 else 4099) for q in range(n)]
    elif layout == "unaligned":
        blocks = [(q * 4097 + q, 4097) for q in range(n)]
    else:
        counts = [(40961 * (q + 3)) % 15001 + 1 for q in range(n)]
        blocks = [(sum(counts[:q]), counts[q]) for q in range(n)]
    check_general(RSV, n, 0, es, vec=True, vblocks=blocks)
    check_general(RSV, n, 0, es, vec=False, vblocks=blocks)


@pytest.mark.parametrize("tile_vecs,count", [(1, 5), (1, 4099), (3, 33333), (64, 4099), (64, 300007), (4096, 300007)])
@pytest.mark.parametrize("es", [1, 2, 4, 8])
def test_ipc_tiled_block_shares_in_bounds_and_exact_cover(tile_vecs, es, count):
    """HCCL_AMD_IPC_TILE_KIB: block b's share is the tiles b, b + B, ... of the piece instead of one window; every kind
    stays in bounds, covers each element once per phase, and block b keeps the same coordinates in every round."""
    tile = tile_vecs * (16 // es)
    for kind, n in ((AR, 2), (AR, 8), (RS, 3), (RED, 4)):
        check(kind, n, count, es, vec=True, root=n - 1, tile=tile)
    check(ARBAL, 4, count, es, vec=True, group=8, tile=tile)
    for kind in (AR1, RED1):
        check_general(kind, 3, count, es, vec=True, root=2, tile=tile)
    check_general(ARMC, 4, count, es, vec=True, o6=True, tile=tile)
    check_general(RS, 8, count, es, vec=False, o6=True, tile=tile)


def test_ipc_tiled_multi_round():
    n, count = 2, (36 << 20) + 11  # fp32: 3 rounds of 16 Mi elements
    check(AR, n, count, 4, vec=True, root=1, tile=4096)
