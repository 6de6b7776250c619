"""Host-side model of the one-sided kernel's LL form (ipc.cc RunIpcPlan / LlIpcBlocks, ipc_kernel_body.h LlOneShot):
for every rank count, element size and count up to HCCL_AMD_IPC_LL_BYTES' 64 KiB, the blocks' windows partition the
call, their LL words partition its words (no two blocks ever store or poll one word), every word lies inside its LL
slot, every unpacked word inside the unpack area, and the partial last word reads no byte past the input. CPU only:
the GPU tests (tests/test_gpu_small_ipc.py) check the bits."""
import pytest

LL_MAX = 64 << 10                 # kIpcLlMaxBytes
SLOT_BYTES = 2 * LL_MAX           # kIpcLlSlotBytes
MAX_RANKS = 16                    # kIpcMaxRanks
UNPACK_BYTES = MAX_RANKS * (LL_MAX + 256)  # kIpcLlUnpackBytes
LOOPBACK_BLOCK_CAP = 128          # kIpcBlocks


def ll_blocks(n, nbytes, rhd=False):
    """ipc.cc LlIpcBlocks."""
    items = max(n - 1, 1) * ((nbytes + 3) // 4)
    per = 256 if rhd else 512
    return min(128, max(2, (items + per - 1) // per))


def windows(count, es, blocks):
    v = 16 // es
    piece = max(v, (count + v - 1) // v * v)                      # one-shot: the whole call, one round
    block_elems = ((piece + blocks - 1) // blocks + v - 1) // v * v
    out = []
    for b in range(blocks):
        lo = min(count, b * block_elems)
        out.append((lo, min(count, lo + block_elems)))
    return piece, out


def check(n, es, count, blocks):
    nbytes = count * es
    assert nbytes <= LL_MAX
    piece, wins = windows(count, es, blocks)
    covered = 0
    words_seen = set()
    n_words = (nbytes + 3) // 4
    slot_words = piece * es // 4
    assert piece * es % 16 == 0
    for lo, hi in wins:
        assert lo == covered or lo == hi == count
        covered = max(covered, hi)
        wlo, whi = lo * es // 4, ((hi * es + 3) // 4 if hi > lo else lo * es // 4)  # LlOneShot
        if lo == hi:
            assert wlo == whi
            continue
        assert lo * es % 16 == 0                                   # windows start on 16-B boundaries
        ws = set(range(wlo, whi))
        assert not (ws & words_seen)                               # no word shared by two blocks
        words_seen |= ws
        assert whi * 8 <= SLOT_BYTES                               # LlWord inside the slot
        for q in range(n):
            assert (q * slot_words + whi) * 4 <= UNPACK_BYTES      # unpack store inside the area
        assert whi * 4 <= piece * es                               # unpacked words inside slot q's fold range
        # LoadWord: a word past the input's end reads nothing beyond it (only bytes o + i < nbytes)
        assert min(nbytes, whi * 4) <= nbytes
    assert covered == count
    assert words_seen == set(range(n_words))


@pytest.mark.parametrize("n", [2, 3, 4, 5, 8, 16])
@pytest.mark.parametrize("es", [1, 2, 4, 8])
@pytest.mark.parametrize("nbytes", [1, 3, 4, 5, 15, 16, 17, 1000, 1024, 4097, 16384, 32771, 65535, 65536])
def test_ll_windows_words_and_areas(n, es, nbytes):
    count = max(1, nbytes // es)
    if count * es > LL_MAX:
        return
    computed = ll_blocks(n, count * es)
    for blocks in sorted({computed, ll_blocks(n, count * es, rhd=True), 1, 3, 128}):
        check(n, es, count, blocks)


def test_ll_block_rule():
    """About two polled words per thread of 256 (RHD's order: one), never fewer than two blocks nor more than 128:
    1 KiB at n = 2 is two blocks, 64 KiB at n = 2 thirty-two (RHD sixty-four)."""
    assert ll_blocks(2, 1024) == 2
    assert ll_blocks(2, 4096) == 2 and ll_blocks(2, 4096, rhd=True) == 4
    assert ll_blocks(2, 65536) == 32 and ll_blocks(2, 65536, rhd=True) == 64
    assert ll_blocks(8, 65536) == 128
    assert all(2 <= ll_blocks(n, b, r) <= 128 for n in range(2, 17) for b in range(1, LL_MAX + 1, 511)
               for r in (False, True))


@pytest.mark.parametrize("n", [2, 3, 8, 16])
@pytest.mark.parametrize("nw", [0, 1, 5, 64, 257, 16384])
@pytest.mark.parametrize("threads", [256, 512])
def test_push_items_cover_every_peer_word_once(n, nw, threads):
    """LlOneShot's push (ipc_kernel_body.h): a ReduceScatter's items are (peer, word) pairs, the word fastest, dealt to
    the block's threads in batches of kLlBatch x threads; every peer's every word of the window is stored exactly once,
    and the item index stays inside 32 bits. A one-shot's items are its words, each stored to every peer."""
    K = 8  # kLlBatch
    me, wlo = n - 1, 1000
    for per_dest in (True, False):
        items = (n - 1) * nw if per_dest else nw
        assert items < 2 ** 32 - K * threads
        stored = []
        for t in range(threads):
            base = t
            while base < items:
                for k in range(K):
                    i = base + k * threads
                    if i >= items:
                        continue
                    c = (me + 1 + i // nw) % n if per_dest else me
                    w = wlo + (i % nw if per_dest else i)
                    if per_dest:
                        stored.append((c, w))
                    else:
                        stored.extend(((me + j) % n, w) for j in range(1, n))
                base += K * threads
        want = [((me + j) % n, wlo + x) for j in range(1, n) for x in range(nw)]
        assert sorted(stored) == sorted(want)
        assert all(c != me for c, _ in stored)

