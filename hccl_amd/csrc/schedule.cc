// schedule.cc — schedule IR generators (see schedule.h).
//
// Association orders, per element, with "acc = src (op) acc" as in LocalReduce:
//   one-shot AllReduce, mesh ReduceScatter, Reduce   O1: acc = x_me, then x_r for r ascending, r != me
//       ins_temp_all_reduce_mesh_1D_one_shot.cc:211-226, ins_temp_reduce_scatter_mesh_1D.cc:165-203,
//       reduce_mesh_1D.cc:232-246, reduce_mesh_1D_two_shot.cc:226-247
//   two-shot AllReduce                               O2: acc = x_0, then x_1 .. x_{n-1}
//       ins_temp_all_reduce_mesh_1D_two_shot.cc:312-338
//   rings (build-side; the reference has no ring AllReduce template): R arc-disjoint Hamiltonian cycles, part k on
//       ring k; chunk at position c: acc = x_{cyc[c+1]}, then x_{cyc[c+2]} .. x_{cyc[c]}
//   RHD (docs/zh/user_guide/coll_algo_intro/RHD.md)  pairwise tree, partner = rank ^ d, d = n/2, n/4, .., 1
//   NHR AllReduce                                    O5: ins_temp_all_reduce_nhr.cc:230-301, 390-482
//
// Data movement: a rank's data leaves it through SEND/RECV records grouped into one RCCL group per pipeline step;
// every schedule is cut into pieces ("pipelining granule") so that the transfer of piece t+1 overlaps the reduce
// of piece t, and the staging ("CCL buffer", SCRATCH) holds only a bounded number of pieces. The executor derives
// every cross-stream dependency from the byte ranges the records touch, so the generators only have to emit a
// correct program order.
#include "schedule.h"

#include <algorithm>

namespace hccl_amd {

namespace {

constexpr uint64_t kAlignBytes = 128;  // HCCL_MIN_SLICE_ALIGN, alg_template_base.h:34
constexpr uint64_t kOneShotMaxBytes = 8ull << 20;

struct Ref {
    int32_t buf;
    uint64_t off;
};

class Builder {
public:
    std::vector<HcclAmdIrOp> ops;
    uint64_t scratchHigh = 0;
    int32_t group = 0;
    // Element offset added to every INPUT / OUTPUT reference: a generator written for [0, count) then runs one
    // executor loop [ioBase, ioBase + count) of the reference's OrchestrateLoop.
    uint64_t ioBase = 0;

    void Copy(Ref dst, Ref src, uint64_t count)
    {
        if (count == 0) return;
        HcclAmdIrOp o = Blank(HCCL_AMD_IR_COPY, count);
        SetDst(o, dst, count);
        AddSrc(o, src, count);
        ops.push_back(o);
    }
    void Reduce(Ref dst, const std::vector<Ref>& srcs, uint64_t count)
    {
        if (count == 0) return;
        HcclAmdIrOp o = Blank(HCCL_AMD_IR_REDUCE, count);
        SetDst(o, dst, count);
        for (const Ref& s : srcs) AddSrc(o, s, count);
        ops.push_back(o);
    }
    void Send(uint32_t peer, Ref src, uint64_t count)
    {
        if (count == 0) return;
        HcclAmdIrOp o = Blank(HCCL_AMD_IR_SEND, count);
        o.peer = static_cast<int32_t>(peer);
        o.group = group;
        AddSrc(o, src, count);
        ops.push_back(o);
    }
    void Recv(uint32_t peer, Ref dst, uint64_t count)
    {
        if (count == 0) return;
        HcclAmdIrOp o = Blank(HCCL_AMD_IR_RECV, count);
        o.peer = static_cast<int32_t>(peer);
        o.group = group;
        SetDst(o, dst, count);
        ops.push_back(o);
    }
    void EndGroup() { group++; }

private:
    static HcclAmdIrOp Blank(int32_t kind, uint64_t count)
    {
        HcclAmdIrOp o{};
        o.kind = kind;
        o.peer = -1;
        o.nsrc = 0;
        o.group = -1;
        o.count = count;
        o.dstBuf = -1;
        for (int i = 0; i < HCCL_AMD_IR_MAX_SRC; ++i) o.srcBuf[i] = -1;
        return o;
    }
    void Track(Ref r, uint64_t count)
    {
        if (r.buf == HCCL_AMD_BUF_SCRATCH) scratchHigh = std::max(scratchHigh, r.off + count);
    }
    uint64_t Base(Ref r) const { return r.buf == HCCL_AMD_BUF_SCRATCH ? r.off : r.off + ioBase; }
    void SetDst(HcclAmdIrOp& o, Ref r, uint64_t count)
    {
        o.dstBuf = r.buf;
        o.dstOff = Base(r);
        Track(r, count);
    }
    void AddSrc(HcclAmdIrOp& o, Ref r, uint64_t count)
    {
        o.srcBuf[o.nsrc] = r.buf;
        o.srcOff[o.nsrc] = Base(r);
        o.nsrc++;
        Track(r, count);
    }
};

uint64_t AlignUp(uint64_t v, uint64_t a) { return (v + a - 1) / a * a; }
uint64_t CeilDiv(uint64_t a, uint64_t b) { return (a + b - 1) / b; }

// A contiguous element range [begin, begin + len).
struct Span {
    uint64_t begin;
    uint64_t len;
};

// Chunk c of n for a buffer of `count` elements: ceil(count / n) rounded up to the 128-B slice alignment
// (two-shot slicing, ins_temp_all_reduce_mesh_1D_two_shot.cc:170-202, with HCCL_MIN_SLICE_ALIGN); trailing chunks
// may be short or empty.
Span Chunk(uint64_t count, uint32_t n, uint32_t c, uint64_t alignElems)
{
    uint64_t sc = AlignUp(CeilDiv(count, n), alignElems);
    uint64_t b = std::min<uint64_t>(count, uint64_t(c) * sc);
    uint64_t e = std::min<uint64_t>(count, b + sc);
    return {b, e - b};
}

// The reference's executor loop (InsV2AllReduceSoleExecutor::OrchestrateLoop,
// ins_v2_all_reduce_sole_executor.cc:160-208; ReduceSoleExecutor, reduce_sole_executor.cc:120-170): at most
// min(transportBound, ccl / scratchMultiple rounded down to 128 B) bytes per loop, and the template slices each loop's
// data on its own. Orders that depend on which rank owns an element (NHR, Reduce two-shot) therefore follow these
// loops. ccl = HCCL_BUFFSIZE (the reference's simulator and default: 200 MB).
constexpr uint64_t kUbMaxDataSize = 256ull << 20;  // UB_MAX_DATA_SIZE, alg_param.h:37

uint64_t RefLoopElems(const ScheduleParams& p, uint64_t transportBoundBytes, uint64_t scratchMultiple)
{
    const uint64_t ccl = p.cclBytes;
    uint64_t bytes = transportBoundBytes;
    if (scratchMultiple != 0) bytes = std::min(bytes, ccl / scratchMultiple / kAlignBytes * kAlignBytes);
    return std::max<uint64_t>(1, bytes / p.elemSize);
}

// Runs gen(loopParams) once per executor loop, with the builder's I/O base at the loop's first element.
template <class Gen>
void ForEachRefLoop(const ScheduleParams& p, Builder& b, uint64_t loopElems, Gen gen)
{
    for (uint64_t off = 0; off < p.count; off += loopElems) {
        ScheduleParams lp = p;
        lp.count = std::min(loopElems, p.count - off);
        b.ioBase = off;
        gen(lp);
    }
    b.ioBase = 0;
}

// ReduceMesh1DTwoShot::CalcSlice (reduce_mesh_1D_two_shot.cc:108-131): the first count % n ranks get one element more.
Span BalancedSlice(uint64_t count, uint32_t n, uint32_t c)
{
    const uint64_t base = count / n, rem = count % n;
    return {uint64_t(c) * base + std::min<uint64_t>(c, rem), base + (c < rem ? 1 : 0)};
}

// ReduceNHR::CalcSlice (reduce_nhr.cc:114-138): chunk = RoundUpWithDivisor(bytes, n * elemSize) / n, i.e.
// ceil(count / n) elements; trailing slices short or empty.
Span CeilSlice(uint64_t count, uint32_t n, uint32_t c)
{
    const uint64_t cs = CeilDiv(count, n);
    const uint64_t b = std::min<uint64_t>(count, uint64_t(c) * cs);
    return {b, std::min<uint64_t>(count, b + cs) - b};
}

// InsTempAllReduceNHR::KernelRun (ins_temp_all_reduce_nhr.cc:171-173): floor(count / n), the tail on the last slice.
Span FloorSlice(uint64_t count, uint32_t n, uint32_t c)
{
    const uint64_t se = count / n;
    return c == n - 1 ? Span{uint64_t(c) * se, count - se * (n - 1)} : Span{uint64_t(c) * se, se};
}

// Piece p of a span cut into pieces of pe elements (the last may be short, those past the end are empty).
Span Piece(Span s, uint64_t pe, uint64_t p)
{
    uint64_t b = std::min<uint64_t>(s.len, p * pe);
    uint64_t e = std::min<uint64_t>(s.len, b + pe);
    return {s.begin + b, e - b};
}

// Granule choice: the requested piece size, else about a quarter of the per-peer slice within [256 KiB, 16 MiB];
// then shrunk until `slotsNeeded` staging pieces fit the scratch capacity.
uint64_t PieceElems(const ScheduleParams& p, uint64_t sliceElems, uint64_t slotsNeeded)
{
    const uint64_t es = p.elemSize;
    const uint64_t alignElems = std::max<uint64_t>(1, kAlignBytes / es);
    uint64_t bytes = p.pieceBytes;
    if (bytes == 0) {
        bytes = std::clamp<uint64_t>(sliceElems * es / 4, 256ull << 10, 16ull << 20);
    }
    if (p.scratchCapBytes != 0 && slotsNeeded != 0) {
        uint64_t capPer = p.scratchCapBytes / slotsNeeded;
        capPer = capPer / kAlignBytes * kAlignBytes;
        if (capPer == 0) capPer = kAlignBytes;
        bytes = std::min(bytes, capPer);
    }
    uint64_t pe = std::max<uint64_t>(alignElems, bytes / es / alignElems * alignElems);
    return pe;
}

Ref In(uint64_t off) { return {HCCL_AMD_BUF_INPUT, off}; }
Ref Out(uint64_t off) { return {HCCL_AMD_BUF_OUTPUT, off}; }
Ref Scr(uint64_t off) { return {HCCL_AMD_BUF_SCRATCH, off}; }

// Peer visiting order for mesh steps: me+1, me+2, ... (each rank starts on a different link).
std::vector<uint32_t> PeerOrder(uint32_t n, uint32_t me)
{
    std::vector<uint32_t> v;
    for (uint32_t i = 1; i < n; ++i) v.push_back((me + i) % n);
    return v;
}

// Index of peer q among the n-1 peers in ascending rank order (slot layout of the staging area).
uint32_t PeerSlot(uint32_t q, uint32_t me) { return q < me ? q : q - 1; }

// ------------------------------------------------------------------------------------------- AllReduce

// One-shot (O1): every rank sends its whole input to every peer; each rank folds own + peers ascending.
void AllReduceOneShot(const ScheduleParams& p, Builder& b)
{
    const uint32_t n = p.nRanks, me = p.rank;
    const uint64_t kSlots = 2;
    const uint64_t pe = PieceElems(p, p.count, kSlots * (n - 1));
    const uint64_t np = CeilDiv(p.count, pe);
    auto slot = [&](uint64_t t, uint32_t q) { return Scr(((t % kSlots) * (n - 1) + PeerSlot(q, me)) * pe); };
    for (uint64_t t = 0; t < np; ++t) {
        Span s = Piece({0, p.count}, pe, t);
        for (uint32_t q : PeerOrder(n, me)) {
            b.Send(q, In(s.begin), s.len);
            b.Recv(q, slot(t, q), s.len);
        }
        b.EndGroup();
        std::vector<Ref> srcs{In(s.begin)};
        for (uint32_t q = 0; q < n; ++q) {
            if (q != me) srcs.push_back(slot(t, q));
        }
        b.Reduce(Out(s.begin), srcs, s.len);
    }
}

// Two-shot (O2): mesh reduce-scatter of n chunks, fold of chunk `me` in rank order 0..n-1, mesh all-gather.
// Step t posts the scatter of piece t together with the gather of piece t-2 in one group, so the reduce of piece
// t-1 runs while both transfers are on the links.
void AllReduceTwoShot(const ScheduleParams& p, Builder& b)
{
    const uint32_t n = p.nRanks, me = p.rank;
    const uint64_t alignElems = std::max<uint64_t>(1, kAlignBytes / p.elemSize);
    const uint64_t kSlots = 2;
    const Span mine = Chunk(p.count, n, me, alignElems);
    const uint64_t maxChunk = Chunk(p.count, n, 0, alignElems).len;
    const uint64_t pe = PieceElems(p, maxChunk, kSlots * (n - 1));
    const uint64_t np = std::max<uint64_t>(1, CeilDiv(maxChunk, pe));
    auto slot = [&](uint64_t t, uint32_t q) { return Scr(((t % kSlots) * (n - 1) + PeerSlot(q, me)) * pe); };
    for (uint64_t t = 0; t < np + 2; ++t) {
        if (t < np) {
            Span rs = Piece(mine, pe, t);
            for (uint32_t q : PeerOrder(n, me)) {
                Span out = Piece(Chunk(p.count, n, q, alignElems), pe, t);
                b.Send(q, In(out.begin), out.len);
                b.Recv(q, slot(t, q), rs.len);
            }
        }
        if (t >= 2) {
            uint64_t g = t - 2;
            Span mineP = Piece(mine, pe, g);
            for (uint32_t q : PeerOrder(n, me)) {
                Span theirs = Piece(Chunk(p.count, n, q, alignElems), pe, g);
                b.Send(q, Out(mineP.begin), mineP.len);
                b.Recv(q, Out(theirs.begin), theirs.len);
            }
        }
        b.EndGroup();
        if (t < np) {
            Span rs = Piece(mine, pe, t);
            std::vector<Ref> srcs;
            for (uint32_t q = 0; q < n; ++q) srcs.push_back(q == me ? In(rs.begin) : slot(t, q));
            b.Reduce(Out(rs.begin), srcs, rs.len);
        }
    }
}

// ------------------------------------------------------------------------------------------- MeshChunk (O6)
//
// The reference's MeshChunk templates (ins_temp_all_reduce_mesh_1D_two_shot_mesh_chunk.cc:161-275,
// ins_temp_reduce_scatter_mesh_1D_meshchunk.cc:139-252) cut the chunk that rank t owns into n-1 sub-slices and run
// n-1 steps; in step s every rank write-reduces its raw input of sub-slice i of peer (me - nextNum)'s chunk into
// that peer's CCL buffer, nextNum = s + i + 1, plus one when it reaches n (:207-212 / :200-204). Receiver t thus
// gets sub-slice j at step s from sender t + f(s + j + 1), f(x) = x < n ? x : x + 1. Writes into one receiver are
// serialised step by step: a sender waits for the receiver's ACK of step s+1, which the receiver posts only after all
// of its threads have seen the DATA signals of step s and synchronised (PostSyncInterThreads / PreSyncInterThreads,
// :264-273; SendRecvBatchWriteReduce's handshake, alg_data_trans_wrapper.cc:247-272, 481-514). The CCL buffer starts
// as the receiver's own input (PreCopy), so sub-slice j of owner t is the left fold
//     acc = x_t;  acc = x_{t+o} (op) acc  for o = j+1, ..., n-1, 1, ..., j   (peers by rank offset, mod n)  — O6.
// Here the raw inputs are exchanged into staging slots (as in the two-shot) and every (piece, sub-slice) segment is
// one ordered n-ary fold with that operand order; the data movement granule does not affect the bits.

// Sub-slices of a chunk of `count` elements, AllReduce form (…mesh_chunk.cc:166-183): n-1 slices, the first
// count % (n-1) one element longer.
std::vector<Span> SubSlicesEven(uint64_t count, uint32_t parts)
{
    std::vector<Span> v;
    const uint64_t base = count / parts, big = count % parts;
    uint64_t b = 0;
    for (uint32_t i = 0; i < parts; ++i) {
        const uint64_t len = base + (i < big ? 1 : 0);
        v.push_back({b, len});
        b += len;
    }
    return v;
}

// ReduceScatter form (…meshchunk.cc:155-180): n-2 slices of floor(bytes / (n-1)) rounded down to AICPU_ALIGN_SIZE
// (4 KiB, alg_param.h:91) and the remainder last; the even split when that alignment leaves nothing.
std::vector<Span> SubSlicesRs(uint64_t count, uint32_t parts, uint32_t es)
{
    constexpr uint64_t kAicpuAlign = 4096;
    const uint64_t align = count * es / parts / kAicpuAlign * kAicpuAlign;
    if (parts < 2 || align == 0) return SubSlicesEven(count, parts);
    std::vector<Span> v;
    const uint64_t a = align / es;
    for (uint32_t i = 0; i + 1 < parts; ++i) v.push_back({uint64_t(i) * a, a});
    v.push_back({uint64_t(parts - 1) * a, count - uint64_t(parts - 1) * a});
    return v;
}

// Peers of owner t in the O6 order of sub-slice j (rank offsets j+1 .. n-1, then 1 .. j).
std::vector<uint32_t> O6Peers(uint32_t n, uint32_t t, uint32_t j)
{
    std::vector<uint32_t> v;
    for (uint32_t s = 0; s + 1 < n; ++s) {
        uint32_t x = s + j + 1;
        if (x >= n) x += 1;
        v.push_back((t + x) % n);
    }
    return v;
}

// Emits the folds of one piece [pc.begin, pc.begin + pc.len) of my chunk (chunk-relative coordinates in `subs`):
// own operand at own(e), peer q's at slotOf(q) + (e - pc.begin), result at out(e) — one REDUCE per sub-slice segment.
template <class OwnRef, class OutRef, class SlotRef>
void EmitO6Folds(Builder& b, uint32_t n, uint32_t me, Span pc, const std::vector<Span>& subs, OwnRef own, OutRef out,
                 SlotRef slotOf)
{
    for (uint32_t j = 0; j < subs.size(); ++j) {
        const uint64_t lo = std::max(pc.begin, subs[j].begin);
        const uint64_t hi = std::min(pc.begin + pc.len, subs[j].begin + subs[j].len);
        if (lo >= hi) continue;
        std::vector<Ref> srcs{own(lo)};
        for (uint32_t q : O6Peers(n, me, j)) {
            Ref s = slotOf(q);
            s.off += lo - pc.begin;
            srcs.push_back(s);
        }
        b.Reduce(out(lo), srcs, hi - lo);
    }
}

// AllReduce MeshChunk: executor loops of min(ccl, ccl / 2) (scratch multiple 2, …mesh_chunk.cc:48-55), each sliced
// into n chunks of ceil(count / n) elements (CalcSliceInfoVec :79-97, no 128-B alignment), O6 fold per sub-slice,
// then the mesh all-gather. Pieces of all loops form one pipeline as in the two-shot: step u scatters piece u and
// gathers piece u-2 in one group while piece u-1 is folded.
void AllReduceMeshChunk(const ScheduleParams& p, Builder& b)
{
    const uint32_t n = p.nRanks, me = p.rank;
    const uint64_t loopElems = RefLoopElems(p, p.cclBytes, 2);
    struct Unit {
        uint64_t loopOff, loopCount, t;
    };
    const uint64_t kSlots = 2;
    const uint64_t firstChunk = CeilSlice(std::min(loopElems, p.count), n, 0).len;
    // one staging piece per chunk of a loop when it fits (the loop is already the reference's transfer unit)
    const uint64_t pe = PieceElems(p, 4 * std::max<uint64_t>(1, firstChunk), kSlots * (n - 1));
    std::vector<Unit> units;
    for (uint64_t off = 0; off < p.count; off += loopElems) {
        const uint64_t cnt = std::min(loopElems, p.count - off);
        const uint64_t np = std::max<uint64_t>(1, CeilDiv(CeilSlice(cnt, n, 0).len, pe));
        for (uint64_t t = 0; t < np; ++t) units.push_back({off, cnt, t});
    }
    auto slot = [&](uint64_t u, uint32_t q) { return Scr(((u % kSlots) * (n - 1) + PeerSlot(q, me)) * pe); };
    auto chunk = [&](const Unit& x, uint32_t c) {
        Span s = CeilSlice(x.loopCount, n, c);
        s.begin += x.loopOff;
        return s;
    };
    const uint64_t nu = units.size();
    for (uint64_t u = 0; u < nu + 2; ++u) {
        if (u < nu) {
            const Unit& x = units[u];
            const Span rs = Piece(chunk(x, me), pe, x.t);
            for (uint32_t q : PeerOrder(n, me)) {
                const Span out = Piece(chunk(x, q), pe, x.t);
                b.Send(q, In(out.begin), out.len);
                b.Recv(q, slot(u, q), rs.len);
            }
        }
        if (u >= 2) {
            const Unit& x = units[u - 2];
            const Span mineP = Piece(chunk(x, me), pe, x.t);
            for (uint32_t q : PeerOrder(n, me)) {
                const Span theirs = Piece(chunk(x, q), pe, x.t);
                b.Send(q, Out(mineP.begin), mineP.len);
                b.Recv(q, Out(theirs.begin), theirs.len);
            }
        }
        b.EndGroup();
        if (u < nu) {
            const Unit& x = units[u];
            const Span mine = chunk(x, me);
            Span pc = Piece({0, mine.len}, pe, x.t);  // chunk-relative
            if (pc.len == 0) continue;
            EmitO6Folds(b, n, me, pc, SubSlicesEven(mine.len, n - 1),
                        [&](uint64_t e) { return In(mine.begin + e); }, [&](uint64_t e) { return Out(mine.begin + e); },
                        [&](uint32_t q) { return slot(u, q); });
        }
    }
}

// ReduceScatter MeshChunk: executor loops of min(ccl - 1 MiB, (ccl - 1 MiB) / (n-1)) (TMP_MEM_RESERVE_SIZE and
// scratch multiple n-1, ins_v2_reduce_scatter_sole_executor.cc:32,160-175; …meshchunk.cc:66-72) over recvCount,
// each block cut into the 4-KiB-aligned sub-slices, O6 fold per sub-slice.
void ReduceScatterMeshChunk(const ScheduleParams& p, Builder& b)
{
    const uint32_t n = p.nRanks, me = p.rank;
    const uint64_t rc = p.count;
    constexpr uint64_t kReserve = 1ull << 20;
    // the reference has no loop at all when HCCL_BUFFSIZE <= 1 MiB (maxDataCountPerLoop == 0 → HCCL_E_INTERNAL);
    // here the whole CCL size is used then
    const uint64_t tmp = p.cclBytes > kReserve ? p.cclBytes - kReserve : p.cclBytes;
    const uint64_t loopBytes = std::min(tmp, tmp / (n - 1) / kAlignBytes * kAlignBytes);
    const uint64_t loopElems = std::max<uint64_t>(1, loopBytes / p.elemSize);
    const uint64_t kSlots = 2;
    const uint64_t pe = PieceElems(p, std::min(rc, loopElems), kSlots * (n - 1));
    auto slot = [&](uint64_t u, uint32_t q) { return Scr(((u % kSlots) * (n - 1) + PeerSlot(q, me)) * pe); };
    uint64_t u = 0;
    for (uint64_t off = 0; off < rc; off += loopElems) {
        const uint64_t cnt = std::min(loopElems, rc - off);
        const std::vector<Span> subs = SubSlicesRs(cnt, n - 1, p.elemSize);
        const uint64_t np = std::max<uint64_t>(1, CeilDiv(cnt, pe));
        for (uint64_t t = 0; t < np; ++t, ++u) {
            const Span pc = Piece({0, cnt}, pe, t);  // loop-relative
            for (uint32_t q : PeerOrder(n, me)) {
                b.Send(q, In(uint64_t(q) * rc + off + pc.begin), pc.len);
                b.Recv(q, slot(u, q), pc.len);
            }
            b.EndGroup();
            EmitO6Folds(b, n, me, pc, subs, [&](uint64_t e) { return In(uint64_t(me) * rc + off + e); },
                        [&](uint64_t e) { return Out(off + e); }, [&](uint32_t q) { return slot(u, q); });
        }
    }
}

// ------------------------------------------------------------------------------------------- rings over xGMI
//
// xGMI is point to point: a single directed ring moves every byte over ONE link per rank, 1/7 of what an 8-GPU
// node offers. The ring schedules therefore run R arc-disjoint directed Hamiltonian cycles at once (RingTable):
// the complete digraph on n ranks decomposes into n-1 of them for n != 4, 6 (Tillson), so at n = 8 seven rings use
// all seven outgoing and incoming links of every GPU. The buffer is split into R parts; part k travels around ring
// k. Inside a ring, ranks are addressed by their position v on the cycle (rank = cycle[v]), which is the reference's
// ring neighbour convention prev = v-1, next = v+1 (scatter_ring.cc:186-187) applied to the cycle.

// The rings for n ranks (every rank computes the same table): found by search and checked in tests/test_schedules.py
// (each is a Hamiltonian cycle, no arc is used twice); n > 8: the rotations v -> v + k with gcd(k, n) = 1.
}  // namespace

std::vector<std::vector<uint32_t>> RingTable(uint32_t n)
{
    switch (n) {
        case 1: return {{0}};
        case 2: return {{0, 1}};
        case 3: return {{0, 1, 2}, {0, 2, 1}};
        case 4: return {{0, 1, 3, 2}, {0, 2, 3, 1}};
        case 5: return {{0, 3, 1, 2, 4}, {0, 1, 4, 3, 2}, {0, 4, 2, 1, 3}, {0, 2, 3, 4, 1}};
        case 6: return {{0, 3, 1, 2, 5, 4}, {0, 4, 5, 2, 1, 3}, {0, 2, 3, 4, 1, 5}, {0, 5, 1, 4, 3, 2}};
        case 7:
            return {{0, 5, 1, 6, 4, 3, 2}, {0, 2, 3, 6, 1, 4, 5}, {0, 3, 1, 2, 5, 4, 6}, {0, 4, 1, 5, 2, 6, 3},
                    {0, 1, 3, 5, 6, 2, 4}, {0, 6, 5, 3, 4, 2, 1}};
        case 8:
            return {{0, 5, 6, 3, 7, 2, 1, 4}, {0, 4, 2, 3, 5, 7, 1, 6}, {0, 3, 2, 7, 5, 4, 6, 1},
                    {0, 7, 6, 2, 4, 1, 5, 3}, {0, 2, 6, 5, 1, 3, 4, 7}, {0, 1, 7, 3, 6, 4, 5, 2},
                    {0, 6, 7, 4, 3, 1, 2, 5}};
        default: {
            std::vector<std::vector<uint32_t>> t;
            for (uint32_t k = 1; k < n; ++k) {
                uint32_t a = k, bb = n;
                while (bb != 0) {
                    const uint32_t r = a % bb;
                    a = bb;
                    bb = r;
                }
                if (a != 1) continue;
                std::vector<uint32_t> c;
                for (uint32_t v = 0; v < n; ++v) c.push_back(uint32_t((uint64_t(v) * k) % n));
                t.push_back(c);
            }
            return t;
        }
    }
}

namespace {

// One ring of the table as seen from rank `me`: its cycle and my position on it.
struct RingView {
    std::vector<uint32_t> cyc;
    uint32_t pos;
    uint32_t At(int64_t v) const
    {
        const int64_t n = int64_t(cyc.size());
        return cyc[size_t(((v % n) + n) % n)];
    }
    uint32_t Next() const { return At(int64_t(pos) + 1); }
    uint32_t Prev() const { return At(int64_t(pos) - 1); }
};

// How many of the rings a call uses. Every ring adds two messages per rank and step, about 1 us of host time each on
// the executor (profiles/r02_rccl_selfloop_latency*.jsonl), and spreads the transfer over one more link (1 MiB takes
// 13.65 us at 76.8 GB/s). The AllReduce (2(n-1) steps, 2(n-1)/n x bytes moved), the ReduceScatter and the AllGather
// ((n-1) steps, (n-1)/n x the input / output bytes) all balance at R^2 = 13.65 x MiB / (2n): the largest R with
// R^2 x 2n x 1 MiB <= 13.65 x bytes, at least 1 (one ring up to ~4.7 MiB at n = 8, all seven from ~57 MiB). `bytes` is
// the AllReduce buffer, the ReduceScatter input or the AllGather output of one rank.
std::vector<RingView> Rings(uint32_t n, uint32_t me, uint64_t bytes)
{
    std::vector<std::vector<uint32_t>> table = RingTable(n);
    size_t rings = 1;
    while (rings < table.size() &&
           double(rings + 1) * double(rings + 1) * 2.0 * n * double(1u << 20) <= 13.65 * double(bytes)) {
        ++rings;
    }
    table.resize(std::min(table.size(), rings));
    std::vector<RingView> v;
    for (auto& c : table) {
        RingView r{c, 0};
        for (uint32_t i = 0; i < n; ++i) {
            if (c[i] == me) r.pos = i;
        }
        v.push_back(r);
    }
    return v;
}

// Part k of R of a buffer of `count` elements: ceil(count / R) rounded up to 128 B; trailing parts short or empty.
Span RingPart(uint64_t count, uint32_t R, uint32_t k, uint64_t alignElems) { return Chunk(count, R, k, alignElems); }

// AllReduce over R rings: in part k, position v owns chunk v; n-1 reduce-scatter steps (position v receives chunk
// v-s-2 from v-1 and folds it into its own copy: acc = travelling partial (src) (op) own input), then n-1 all-gather
// steps. Every step posts all rings' transfers in one group; pieces pipeline the steps.
void AllReduceRing(const ScheduleParams& p, Builder& b)
{
    const uint32_t n = p.nRanks, me = p.rank;
    const uint64_t alignElems = std::max<uint64_t>(1, kAlignBytes / p.elemSize);
    const std::vector<RingView> rings = Rings(n, me, p.count * p.elemSize);
    const uint32_t R = static_cast<uint32_t>(rings.size());
    const uint64_t kSlots = 4;
    const Span part0 = RingPart(p.count, R, 0, alignElems);
    const uint64_t maxChunk = Chunk(part0.len, n, 0, alignElems).len;
    const uint64_t pe = PieceElems(p, maxChunk, kSlots * R);
    const uint64_t np = std::max<uint64_t>(1, CeilDiv(maxChunk, pe));
    auto chunkOf = [&](uint32_t k, uint32_t c) {
        const Span part = RingPart(p.count, R, k, alignElems);
        Span ch = Chunk(part.len, n, c, alignElems);
        ch.begin += part.begin;
        return ch;
    };
    uint64_t unit = 0;
    for (uint32_t s = 0; s + 1 < n; ++s) {
        for (uint64_t t = 0; t < np; ++t, ++unit) {
            for (uint32_t k = 0; k < R; ++k) {
                const RingView& r = rings[k];
                const uint32_t cs = (r.pos + 2 * n - s - 1) % n;
                const uint32_t cr = (r.pos + 2 * n - s - 2) % n;
                const Span snd = Piece(chunkOf(k, cs), pe, t);
                const Span rcv = Piece(chunkOf(k, cr), pe, t);
                b.Send(r.Next(), s == 0 ? In(snd.begin) : Out(snd.begin), snd.len);
                b.Recv(r.Prev(), Scr(((unit % kSlots) * R + k) * pe), rcv.len);
            }
            b.EndGroup();
            for (uint32_t k = 0; k < R; ++k) {
                const uint32_t cr = (rings[k].pos + 2 * n - s - 2) % n;
                const Span rcv = Piece(chunkOf(k, cr), pe, t);
                b.Reduce(Out(rcv.begin), {In(rcv.begin), Scr(((unit % kSlots) * R + k) * pe)}, rcv.len);
            }
        }
    }
    // All-gather: received chunks land in recvBuf directly, so no staging bounds the granule, and there is no fold to
    // pipeline against: every step moves whole chunks on all R rings at once (one transport group per step instead
    // of one per staging piece, which saves a group launch per piece; tools/executor_overlap_model.py).
    for (uint32_t s = 0; s + 1 < n; ++s) {
        for (uint32_t k = 0; k < R; ++k) {
            const RingView& r = rings[k];
            const uint32_t cs = (r.pos + n - s) % n;
            const uint32_t cr = (r.pos + 2 * n - s - 1) % n;
            const Span snd = chunkOf(k, cs);
            const Span rcv = chunkOf(k, cr);
            b.Send(r.Next(), Out(snd.begin), snd.len);
            b.Recv(r.Prev(), Out(rcv.begin), rcv.len);
        }
        b.EndGroup();
    }
}

// Recursive halving (reduce-scatter) then recursive doubling (all-gather), power-of-two n = 2^m
// (docs/zh/user_guide/coll_algo_intro/RHD.md). One RHD instance uses one link per step (partner = rank ^ d), 3 of an
// 8-GPU node's 7. The ranks of a power-of-two world are the vectors of GF(2)^m and the 7 XOR matchings r <-> r ^ v
// (v != 0) partition its links, so the schedule runs up to n-1 instances at once (RhdInstances: fewer for small
// calls), one per part of the buffer: instance j
// relabels ranks by the linear map whose step-s partner vector is alpha^(s+j) in GF(2^m) (alpha primitive). At every
// step the instances' vectors alpha^(s+j), j = 0..n-2, are all the nonzero vectors: every link carries exactly one.
// Inside instance j the classic RHD runs on virtual ranks: region = virtual chunk range [lo, hi); at virtual distance
// d the rank keeps the half selected by bit d of its virtual rank and exchanges the other half with its partner.
// It ends with virtual rank v owning chunk v of the part.

// Multiplication in GF(2^m) modulo a primitive polynomial (m <= 4: x^2+x+1, x^3+x+1, x^4+x+1).
uint32_t Gf2Mul(uint32_t a, uint32_t b, uint32_t m)
{
    static const uint32_t kPoly[5] = {0, 0x3, 0x7, 0xB, 0x13};
    uint32_t r = 0;
    for (uint32_t i = 0; i < m; ++i) {
        if ((b >> i) & 1u) r ^= a << i;
    }
    for (uint32_t i = 2 * m; i-- > m;) {
        if ((r >> i) & 1u) r ^= kPoly[m] << (i - m);
    }
    return r;
}

}  // namespace

std::vector<std::vector<uint32_t>> RhdTable(uint32_t n)
{
    // returns, per instance, virt->real rank (index = virtual rank)
    uint32_t m = 0;
    while ((1u << m) < n) ++m;
    if ((1u << m) != n || m > 4) return {};
    if (m == 0) return {{0}};
    std::vector<std::vector<uint32_t>> t;
    for (uint32_t j = 0; j + 1 < n; ++j) {
        // partner vector of step s (virtual bit m-1-s) is alpha^(s+j), alpha = 2
        std::vector<uint32_t> vec(m);
        for (uint32_t s2 = 0; s2 < m; ++s2) {
            uint32_t x = 1;
            for (uint32_t k = 0; k < s2 + j; ++k) x = Gf2Mul(x, 2, m);
            vec[s2] = x;
        }
        std::vector<uint32_t> real(n);
        for (uint32_t v = 0; v < n; ++v) {
            uint32_t r = 0;
            for (uint32_t s2 = 0; s2 < m; ++s2) {
                if ((v >> (m - 1 - s2)) & 1u) r ^= vec[s2];
            }
            real[v] = r;
        }
        t.push_back(real);
    }
    return t;
}

// How many of the n-1 instances a call of `bytes` per rank runs. Every instance adds one message per rank and step
// (6 steps at n = 8), and on the executor each message costs host time whatever its size: about 10 us per transport
// group plus 1 us per message (RCCL self-loop programs, profiles/r02_rccl_selfloop_latency.jsonl). What an instance
// buys is link bandwidth: R instances spread 2 (n-1)/n x bytes over R links at 76.8 GB/s each. With 12 us per extra
// instance against 22.8 us per MiB / R of transfer, the best R is about sqrt(2 x bytes / 1 MiB): one instance up to
// 1 MiB (C5's latency range), all seven from 24.5 MiB. Ranks agree: it depends on the call's arguments only.
uint32_t RhdInstances(uint32_t n, uint64_t bytes)
{
    const uint32_t most = n > 1 ? n - 1 : 1;
    uint32_t r = 1;
    while (r < most && uint64_t(r + 1) * (r + 1) * (1ull << 20) <= 2 * bytes) ++r;
    return r;
}

namespace {

void AllReduceRhd(const ScheduleParams& p, Builder& b)
{
    const uint32_t n = p.nRanks, me = p.rank;
    const uint64_t alignElems = std::max<uint64_t>(1, kAlignBytes / p.elemSize);
    std::vector<std::vector<uint32_t>> table = RhdTable(n);
    table.resize(std::min<size_t>(table.size(), RhdInstances(n, p.count * p.elemSize)));
    const uint32_t R = static_cast<uint32_t>(table.size());
    struct Inst {
        std::vector<uint32_t> real;
        uint32_t v;  // my virtual rank
        Span part;
        uint32_t lo, hi;
    };
    std::vector<Inst> inst(R);
    for (uint32_t j = 0; j < R; ++j) {
        inst[j].real = table[j];
        for (uint32_t v = 0; v < n; ++v) {
            if (table[j][v] == me) inst[j].v = v;
        }
        inst[j].part = Chunk(p.count, R, j, alignElems);
        inst[j].lo = 0;
        inst[j].hi = n;
    }
    auto range = [&](const Inst& I, uint32_t lo, uint32_t hi) {
        Span a = Chunk(I.part.len, n, lo, alignElems);
        Span z = Chunk(I.part.len, n, hi - 1, alignElems);
        return Span{I.part.begin + a.begin, z.begin + z.len - a.begin};
    };
    const uint64_t kSlots = 4;
    const uint64_t pe = PieceElems(p, range(inst[0], 0, n / 2).len, kSlots * R);
    uint64_t unit = 0;
    bool first = true;
    for (uint32_t d = n / 2; d >= 1; d /= 2) {
        // the piece count is the same on every rank (partners of different instances share groups): the widest
        // half any rank can hold at this distance is the first d chunks of part 0
        const uint64_t np = std::max<uint64_t>(1, CeilDiv(range(inst[0], 0, d).len, pe));
        std::vector<Span> keep(R), give(R);
        for (uint32_t j = 0; j < R; ++j) {
            const Inst& I = inst[j];
            const uint32_t mid = I.lo + d;
            const bool keepLow = (I.v & d) == 0;
            keep[j] = keepLow ? range(I, I.lo, mid) : range(I, mid, I.hi);
            give[j] = keepLow ? range(I, mid, I.hi) : range(I, I.lo, mid);
        }
        for (uint64_t t = 0; t < np; ++t, ++unit) {
            for (uint32_t j = 0; j < R; ++j) {
                const uint32_t partner = inst[j].real[inst[j].v ^ d];
                const Span g = Piece(give[j], pe, t);
                const Span k = Piece(keep[j], pe, t);
                b.Send(partner, first ? In(g.begin) : Out(g.begin), g.len);
                b.Recv(partner, Scr(((unit % kSlots) * R + j) * pe), k.len);
            }
            b.EndGroup();
            for (uint32_t j = 0; j < R; ++j) {
                const Span k = Piece(keep[j], pe, t);
                b.Reduce(Out(k.begin), {first ? In(k.begin) : Out(k.begin), Scr(((unit % kSlots) * R + j) * pe)},
                         k.len);
            }
        }
        for (Inst& I : inst) {
            const uint32_t mid = I.lo + d;
            if ((I.v & d) == 0) {
                I.hi = mid;
            } else {
                I.lo = mid;
            }
        }
        first = false;
        if (d == 1) break;
    }
    // Recursive doubling: the exchanged halves land in recvBuf directly (no staging, no fold), so every step moves
    // whole regions in one transport group (as the ring's all-gather).
    for (uint32_t d = 1; d < n; d *= 2) {
        std::vector<Span> mine(R), theirs(R);
        std::vector<uint32_t> plo(R);
        for (uint32_t j = 0; j < R; ++j) {
            const Inst& I = inst[j];
            // my region is [lo, lo + d) virtual chunks; the partner's is the adjacent block of d chunks
            plo[j] = (I.v & d) == 0 ? I.lo + d : I.lo - d;
            mine[j] = range(I, I.lo, I.lo + d);
            theirs[j] = range(I, plo[j], plo[j] + d);
        }
        for (uint32_t j = 0; j < R; ++j) {
            const uint32_t partner = inst[j].real[inst[j].v ^ d];
            b.Send(partner, Out(mine[j].begin), mine[j].len);
            b.Recv(partner, Out(theirs[j].begin), theirs[j].len);
        }
        b.EndGroup();
        for (uint32_t j = 0; j < R; ++j) inst[j].lo = std::min(inst[j].lo, plo[j]);
    }
}

// NHR (ins_temp_all_reduce_nhr.cc:171-173, 230-369, 390-482): ceil(log2 n) reduce-scatter steps in which rank r
// sends slices r-2^k, r-2^k-2^(k+1), ... to r-2^k and receives slices r, r-2^(k+1), ... from r+2^k, folding each as
// receiver partial (dst) (op) sender partial (src); then the mirrored all-gather. Slices are floor(count/n) with the
// tail on the last slice. The reference works in its CCL buffer (PreCopy / PostCopy); here recvBuf is the working
// buffer, which gives the same per-element order.
struct NhrStep {
    uint32_t to, from;
    std::vector<uint32_t> tx, rx;
};

std::vector<NhrStep> NhrSteps(uint32_t n, uint32_t me, bool gather)
{
    uint32_t nSteps = 0;
    for (uint32_t t = n - 1; t != 0; t >>= 1) nSteps++;
    std::vector<NhrStep> out(nSteps);
    for (uint32_t step = 0; step < nSteps; ++step) {
        NhrStep& st = out[step];
        uint32_t nSlices, delta, tx, rx;
        if (!gather) {
            const uint32_t dr = 1u << step;
            st.to = (me + n - dr) % n;
            st.from = (me + dr) % n;
            nSlices = (n - 1 + (1u << step)) / (1u << (step + 1));
            delta = 1u << (step + 1);
            tx = st.to;
            rx = me;
        } else {
            const uint32_t dr = 1u << (nSteps - 1 - step);
            st.to = (me + dr) % n;
            st.from = (me + n - dr) % n;
            nSlices = (n - 1 + dr) / (1u << (nSteps - step));
            delta = 1u << (nSteps - step);
            tx = me;
            rx = (me + n - dr) % n;
        }
        for (uint32_t i = 0; i < nSlices; ++i) {
            st.tx.push_back(tx);
            st.rx.push_back(rx);
            tx = (tx + n - delta % n) % n;
            rx = (rx + n - delta % n) % n;
        }
    }
    return out;
}

void AllReduceNhrLoop(const ScheduleParams& p, Builder& b)
{
    const uint32_t n = p.nRanks, me = p.rank;
    auto slice = [&](uint32_t i) { return FloorSlice(p.count, n, i); };
    const uint64_t kSlots = 2;
    const uint64_t maxSlices = (n + 1) / 2;
    const uint64_t tail = slice(n - 1).len;
    const uint64_t pe = PieceElems(p, tail, kSlots * maxSlices);
    const uint64_t np = std::max<uint64_t>(1, CeilDiv(tail, pe));
    b.Copy(Out(0), In(0), p.count);  // PreCopy (ins_temp_all_reduce_nhr.cc PreCopy): the working buffer
    uint64_t unit = 0;
    for (const NhrStep& st : NhrSteps(n, me, false)) {
        for (uint64_t t = 0; t < np; ++t, ++unit) {
            for (size_t i = 0; i < st.tx.size(); ++i) {
                Span s = Piece(slice(st.tx[i]), pe, t);
                b.Send(st.to, Out(s.begin), s.len);
            }
            for (size_t i = 0; i < st.rx.size(); ++i) {
                Span s = Piece(slice(st.rx[i]), pe, t);
                b.Recv(st.from, Scr(((unit % kSlots) * maxSlices + i) * pe), s.len);
            }
            b.EndGroup();
            for (size_t i = 0; i < st.rx.size(); ++i) {
                Span s = Piece(slice(st.rx[i]), pe, t);
                b.Reduce(Out(s.begin), {Out(s.begin), Scr(((unit % kSlots) * maxSlices + i) * pe)}, s.len);
            }
        }
    }
    for (const NhrStep& st : NhrSteps(n, me, true)) {
        for (uint64_t t = 0; t < np; ++t) {
            for (size_t i = 0; i < st.tx.size(); ++i) {
                Span s = Piece(slice(st.tx[i]), pe, t);
                b.Send(st.to, Out(s.begin), s.len);
            }
            for (size_t i = 0; i < st.rx.size(); ++i) {
                Span s = Piece(slice(st.rx[i]), pe, t);
                b.Recv(st.from, Out(s.begin), s.len);
            }
            b.EndGroup();
        }
    }
}

void AllReduceNhr(const ScheduleParams& p, Builder& b)
{
    ForEachRefLoop(p, b, RefLoopElems(p, p.cclBytes, 1), [&](const ScheduleParams& lp) { AllReduceNhrLoop(lp, b); });
}

// NHR ReduceScatter (ins_temp_reduce_scatter_nhr.cc:104-197, 278-397, 407-456): the NHR reduce-scatter steps with the
// ReduceScatter blocks as slices (block i = slice i, whatever the executor loop, so the order does not depend on the
// loop size), write-reduce receiver partial (dst) (op) sender partial (src), then block `me` to recvBuf. Blocks are
// processed in columns of W elements: n working columns in the first ccl bytes of staging, receive slots after them.
void ReduceScatterNhr(const ScheduleParams& p, Builder& b)
{
    const uint32_t n = p.nRanks, me = p.rank;
    const uint64_t rc = p.count;
    const uint64_t alignElems = std::max<uint64_t>(1, kAlignBytes / p.elemSize);
    const uint64_t W = std::min(rc, std::max(alignElems, p.cclBytes / n / p.elemSize / alignElems * alignElems));
    const uint64_t kSlots = 2;
    const uint64_t maxSlices = (n + 1) / 2;
    for (uint64_t col = 0; col < rc; col += W) {
        const uint64_t w = std::min(W, rc - col);
        auto work = [&](uint32_t i, uint64_t off) { return Scr(uint64_t(i) * W + off); };
        ScheduleParams pp = p;
        if (pp.scratchCapBytes != 0) pp.scratchCapBytes -= std::min(pp.scratchCapBytes, n * W * p.elemSize);
        const uint64_t pe = PieceElems(pp, w, kSlots * maxSlices);
        const uint64_t np = std::max<uint64_t>(1, CeilDiv(w, pe));
        auto slot = [&](uint64_t unit, size_t i) { return Scr(n * W + ((unit % kSlots) * maxSlices + i) * pe); };
        for (uint32_t i = 0; i < n; ++i) b.Copy(work(i, 0), In(uint64_t(i) * rc + col), w);  // LocalDataCopy
        uint64_t unit = 0;
        for (const NhrStep& st : NhrSteps(n, me, false)) {
            for (uint64_t t = 0; t < np; ++t, ++unit) {
                const Span s = Piece({0, w}, pe, t);
                for (size_t i = 0; i < st.tx.size(); ++i) b.Send(st.to, work(st.tx[i], s.begin), s.len);
                for (size_t i = 0; i < st.rx.size(); ++i) b.Recv(st.from, slot(unit, i), s.len);
                b.EndGroup();
                for (size_t i = 0; i < st.rx.size(); ++i) {
                    b.Reduce(work(st.rx[i], s.begin), {work(st.rx[i], s.begin), slot(unit, i)}, s.len);
                }
            }
        }
        b.Copy(Out(col), work(me, 0), w);  // PostLocalCopy
    }
}

// ------------------------------------------------------------------------------------------- STRICT tree (O4)

// Order-preserved tree fold. At n <= 8 (MAX_RANK_NUM_FOR_ORDER_PRESERVED, order_preserved_common.h:22), which is every
// single-node case, the reference selects AicpuReduceScatterStrictOrderedMesh / AicpuAllReduceStrictOrderedMesh
// (reduce_scatter_auto_selector.cc:406-413, all_reduce_auto_selector.cc:412-418), i.e. the template
// InsTempReduceScatterOrderPreservedLevel1: its all-to-all puts source s's block for receiver t into t's CCL slot
// CalcOutputIndex(t, s) = (t + s) % n (…order_preserved_level1.cc:176-181, 274-278; own block :196-215), and its
// RunLocalReduce reads virtual index v from slot CalcOutputIndex(v, t) (:322-400), so virtual index = source rank on
// every receiver (tests/test_strict_level1.py restates the template and checks it against this schedule). Above 8
// ranks the Group template folds the same tree (ins_temp_reduce_scatter_order_preserved_group.cc:305-399). The tree:
// while more than one block remains, M = largest power of two below the count and block i >= M is folded into block
// i % M as dst = src (op) dst. n = 8: ((x0+x4)+(x2+x6))+((x1+x5)+(x3+x7)). Rank-independent.
// `blocks` must be writable (staging); the last fold writes `out`.
void EmitTree(Builder& b, const std::vector<Ref>& blocks, Ref out, uint64_t count)
{
    uint32_t remaining = static_cast<uint32_t>(blocks.size());
    if (remaining == 1) {
        b.Copy(out, blocks[0], count);
        return;
    }
    while (remaining > 1) {
        uint32_t m = 1;
        while (m * 2 < remaining) m *= 2;
        for (uint32_t src = m; src < remaining; ++src) {
            const uint32_t dst = src % m;
            b.Reduce(m == 1 ? out : blocks[dst], {blocks[dst], blocks[src]}, count);
        }
        remaining = m;
    }
}

// ReduceScatter in STRICT order: mesh exchange of blocks into per-source staging slots (own block copied in, as
// PreLocalCopy does, :215-232), then the tree fold into recvBuf.
void ReduceScatterTree(const ScheduleParams& p, Builder& b)
{
    const uint32_t n = p.nRanks, me = p.rank;
    const uint64_t rc = p.count;
    const uint64_t kSlots = 2;
    const uint64_t pe = PieceElems(p, rc, kSlots * n);
    const uint64_t np = std::max<uint64_t>(1, CeilDiv(rc, pe));
    auto slot = [&](uint64_t t, uint32_t q) { return Scr(((t % kSlots) * n + q) * pe); };
    for (uint64_t t = 0; t < np; ++t) {
        Span s = Piece({0, rc}, pe, t);
        for (uint32_t q : PeerOrder(n, me)) {
            b.Send(q, In(uint64_t(q) * rc + s.begin), s.len);
            b.Recv(q, slot(t, q), s.len);
        }
        b.EndGroup();
        b.Copy(slot(t, me), In(uint64_t(me) * rc + s.begin), s.len);
        std::vector<Ref> blocks;
        for (uint32_t q = 0; q < n; ++q) blocks.push_back(slot(t, q));
        EmitTree(b, blocks, Out(s.begin), s.len);
    }
}

// AllReduce in STRICT order: the two-shot structure with the tree fold in place of the O2 chain.
void AllReduceTree(const ScheduleParams& p, Builder& b)
{
    const uint32_t n = p.nRanks, me = p.rank;
    const uint64_t alignElems = std::max<uint64_t>(1, kAlignBytes / p.elemSize);
    const uint64_t kSlots = 2;
    const Span mine = Chunk(p.count, n, me, alignElems);
    const uint64_t maxChunk = Chunk(p.count, n, 0, alignElems).len;
    const uint64_t pe = PieceElems(p, maxChunk, kSlots * n);
    const uint64_t np = std::max<uint64_t>(1, CeilDiv(maxChunk, pe));
    auto slot = [&](uint64_t t, uint32_t q) { return Scr(((t % kSlots) * n + q) * pe); };
    for (uint64_t t = 0; t < np + 2; ++t) {
        if (t < np) {
            Span rs = Piece(mine, pe, t);
            for (uint32_t q : PeerOrder(n, me)) {
                Span out = Piece(Chunk(p.count, n, q, alignElems), pe, t);
                b.Send(q, In(out.begin), out.len);
                b.Recv(q, slot(t, q), rs.len);
            }
        }
        if (t >= 2) {
            Span mineP = Piece(mine, pe, t - 2);
            for (uint32_t q : PeerOrder(n, me)) {
                Span theirs = Piece(Chunk(p.count, n, q, alignElems), pe, t - 2);
                b.Send(q, Out(mineP.begin), mineP.len);
                b.Recv(q, Out(theirs.begin), theirs.len);
            }
        }
        b.EndGroup();
        if (t < np) {
            Span rs = Piece(mine, pe, t);
            b.Copy(slot(t, me), In(rs.begin), rs.len);
            std::vector<Ref> blocks;
            for (uint32_t q = 0; q < n; ++q) blocks.push_back(slot(t, q));
            EmitTree(b, blocks, Out(rs.begin), rs.len);
        }
    }
}

// ------------------------------------------------------------------------------------------- ReduceScatter

// Mesh (O1): every rank sends block q to rank q; rank me folds its own block first, then peers ascending
// (ins_temp_reduce_scatter_mesh_1D.cc:138-206). count = recvCount, input block q at q * count.
void ReduceScatterMesh(const ScheduleParams& p, Builder& b)
{
    const uint32_t n = p.nRanks, me = p.rank;
    const uint64_t rc = p.count;
    const uint64_t kSlots = 2;
    const uint64_t pe = PieceElems(p, rc, kSlots * (n - 1));
    const uint64_t np = std::max<uint64_t>(1, CeilDiv(rc, pe));
    auto slot = [&](uint64_t t, uint32_t q) { return Scr(((t % kSlots) * (n - 1) + PeerSlot(q, me)) * pe); };
    for (uint64_t t = 0; t < np; ++t) {
        Span s = Piece({0, rc}, pe, t);
        for (uint32_t q : PeerOrder(n, me)) {
            b.Send(q, In(uint64_t(q) * rc + s.begin), s.len);
            b.Recv(q, slot(t, q), s.len);
        }
        b.EndGroup();
        std::vector<Ref> srcs{In(uint64_t(me) * rc + s.begin)};
        for (uint32_t q = 0; q < n; ++q) {
            if (q != me) srcs.push_back(slot(t, q));
        }
        b.Reduce(Out(s.begin), srcs, s.len);
    }
}

// ReduceScatterV mesh (O1, ins_temp_reduce_scatter_v_mesh_1D.cc:107-146, RunReduceScatterV :148-205): every rank
// writes its input block of peer q, [displs[q], displs[q] + counts[q]), to q; rank me copies its own block to recvBuf
// and folds the peers' copies into it in ascending rank order (PostCopy's LocalReduce loop over tmpRank). Pieces of
// counts[me] are pipelined through two staging slot sets as in the mesh ReduceScatter; the order does not depend on
// them.
void ReduceScatterVMesh(const ScheduleParams& p, Builder& b)
{
    const uint32_t n = p.nRanks, me = p.rank;
    uint64_t widest = 0;
    for (uint32_t q = 0; q < n; ++q) widest = std::max(widest, p.counts[q]);
    const uint64_t kSlots = 2;
    const uint64_t pe = PieceElems(p, std::max<uint64_t>(1, widest), kSlots * (n - 1));
    const uint64_t np = std::max<uint64_t>(1, CeilDiv(widest, pe));  // equal on every rank
    auto slot = [&](uint64_t t, uint32_t q) { return Scr(((t % kSlots) * (n - 1) + PeerSlot(q, me)) * pe); };
    for (uint64_t t = 0; t < np; ++t) {
        const Span mine = Piece({0, p.counts[me]}, pe, t);
        for (uint32_t q : PeerOrder(n, me)) {
            const Span out = Piece({0, p.counts[q]}, pe, t);
            b.Send(q, In(p.displs[q] + out.begin), out.len);
            b.Recv(q, slot(t, q), mine.len);
        }
        b.EndGroup();
        if (mine.len == 0) continue;
        std::vector<Ref> srcs{In(p.displs[me] + mine.begin)};
        for (uint32_t q = 0; q < n; ++q) {
            if (q != me) srcs.push_back(slot(t, q));
        }
        b.Reduce(Out(mine.begin), srcs, mine.len);
    }
}

// Ring reduce-scatter over R rings: every block is split into R parts and part k of every block travels around ring
// k. Step s, position v sends block cycle[v-s-1] (its partial) to v+1 and folds block cycle[v-s-2] received from v-1
// into its own input (acc = travelling partial (src) (op) own input); position v ends with block cycle[v] = its own.
// Partials live in staging until forwarded, the last step writes recvBuf. Rounds of kRound pieces bound the staging.
void ReduceScatterRing(const ScheduleParams& p, Builder& b)
{
    const uint32_t n = p.nRanks, me = p.rank;
    const uint64_t rc = p.count;
    const uint64_t alignElems = std::max<uint64_t>(1, kAlignBytes / p.elemSize);
    const std::vector<RingView> rings = Rings(n, me, rc * n * p.elemSize);
    const uint32_t R = static_cast<uint32_t>(rings.size());
    const uint64_t kRound = 4;
    const uint64_t maxPart = RingPart(rc, R, 0, alignElems).len;
    const uint64_t pe = PieceElems(p, maxPart, 2 * kRound * R);
    const uint64_t np = std::max<uint64_t>(1, CeilDiv(maxPart, pe));
    auto slotAt = [&](uint32_t parity, uint32_t k, uint64_t tr) { return Scr(((parity * R + k) * kRound + tr) * pe); };
    for (uint64_t r0 = 0; r0 < np; r0 += kRound) {
        const uint64_t r1 = std::min(np, r0 + kRound);
        for (uint32_t s = 0; s + 1 < n; ++s) {
            for (uint64_t t = r0; t < r1; ++t) {
                for (uint32_t k = 0; k < R; ++k) {
                    const RingView& r = rings[k];
                    const uint32_t bs = r.At(int64_t(r.pos) - s - 1);
                    const Span piece = Piece(RingPart(rc, R, k, alignElems), pe, t);
                    b.Send(r.Next(), s == 0 ? In(uint64_t(bs) * rc + piece.begin) : slotAt((s + 1) % 2, k, t - r0),
                           piece.len);
                    b.Recv(r.Prev(), slotAt(s % 2, k, t - r0), piece.len);
                }
                b.EndGroup();
                for (uint32_t k = 0; k < R; ++k) {
                    const RingView& r = rings[k];
                    const uint32_t br = r.At(int64_t(r.pos) - s - 2);
                    const Span piece = Piece(RingPart(rc, R, k, alignElems), pe, t);
                    const Ref cur = slotAt(s % 2, k, t - r0);
                    b.Reduce((s + 2 == n) ? Out(piece.begin) : cur, {In(uint64_t(br) * rc + piece.begin), cur},
                             piece.len);
                }
            }
        }
    }
}

// ------------------------------------------------------------------------------------------- Reduce

// Mesh one-shot (O1, me = root): peers send their whole input to the root, which folds own + peers ascending
// (reduce_mesh_1D.cc:136-249). Non-root recvBuf is not touched.
void ReduceOneShot(const ScheduleParams& p, Builder& b)
{
    const uint32_t n = p.nRanks, me = p.rank, root = p.root;
    const uint64_t kSlots = 2;
    const uint64_t pe = PieceElems(p, p.count, kSlots * (n - 1));
    const uint64_t np = CeilDiv(p.count, pe);
    auto slot = [&](uint64_t t, uint32_t q) { return Scr(((t % kSlots) * (n - 1) + PeerSlot(q, root)) * pe); };
    for (uint64_t t = 0; t < np; ++t) {
        Span s = Piece({0, p.count}, pe, t);
        if (me != root) {
            b.Send(root, In(s.begin), s.len);
            b.EndGroup();
            continue;
        }
        for (uint32_t q : PeerOrder(n, me)) b.Recv(q, slot(t, q), s.len);
        b.EndGroup();
        std::vector<Ref> srcs{In(s.begin)};
        for (uint32_t q = 0; q < n; ++q) {
            if (q != me) srcs.push_back(slot(t, q));
        }
        b.Reduce(Out(s.begin), srcs, s.len);
    }
}

// Two-shot: mesh reduce-scatter with O1 per chunk owner (reduce_mesh_1D_two_shot.cc:209-249), then the owners send
// their reduced chunks to the root. Non-roots fold into a staging slot, so their recvBuf is not touched. Slices are
// the template's balanced split of each executor loop (scratch multiple n, transport bound UB_MAX_DATA_SIZE).
void ReduceTwoShotLoop(const ScheduleParams& p, Builder& b)
{
    const uint32_t n = p.nRanks, me = p.rank, root = p.root;
    const uint64_t kSlots = 2;
    const Span mine = BalancedSlice(p.count, n, me);
    const uint64_t maxChunk = BalancedSlice(p.count, n, 0).len;
    // slots: kSlots x (n-1) receive pieces + kSlots reduced pieces (non-root)
    const uint64_t pe = PieceElems(p, maxChunk, kSlots * n);
    const uint64_t np = std::max<uint64_t>(1, CeilDiv(maxChunk, pe));
    auto slot = [&](uint64_t t, uint32_t q) { return Scr(((t % kSlots) * (n - 1) + PeerSlot(q, me)) * pe); };
    auto red = [&](uint64_t t) { return Scr((kSlots * (n - 1) + (t % kSlots)) * pe); };
    for (uint64_t t = 0; t < np + 2; ++t) {
        if (t < np) {
            Span rs = Piece(mine, pe, t);
            for (uint32_t q : PeerOrder(n, me)) {
                Span out = Piece(BalancedSlice(p.count, n, q), pe, t);
                b.Send(q, In(out.begin), out.len);
                b.Recv(q, slot(t, q), rs.len);
            }
        }
        if (t >= 2) {
            uint64_t g = t - 2;
            if (me == root) {
                for (uint32_t q : PeerOrder(n, me)) {
                    Span theirs = Piece(BalancedSlice(p.count, n, q), pe, g);
                    b.Recv(q, Out(theirs.begin), theirs.len);
                }
            } else {
                b.Send(root, red(g), Piece(mine, pe, g).len);
            }
        }
        b.EndGroup();
        if (t < np) {
            Span rs = Piece(mine, pe, t);
            std::vector<Ref> srcs{In(rs.begin)};
            for (uint32_t q = 0; q < n; ++q) {
                if (q != me) srcs.push_back(slot(t, q));
            }
            b.Reduce(me == root ? Out(rs.begin) : red(t), srcs, rs.len);
        }
    }
}

void ReduceTwoShot(const ScheduleParams& p, Builder& b)
{
    ForEachRefLoop(p, b, RefLoopElems(p, kUbMaxDataSize, p.nRanks),
                   [&](const ScheduleParams& lp) { ReduceTwoShotLoop(lp, b); });
}

// NHR Reduce (reduce_nhr.cc:56-106, 164-267, 294-368): the NHR reduce-scatter and all-gather steps over ceil-sized
// slices of each executor loop (scratch multiple 1, transport bound UB_MAX_DATA_SIZE); only the root keeps the result
// (PostCopy :269-292). The working buffer is recvBuf on the root and staging elsewhere (a non-root recvBuf is never
// written); receive slots follow it in staging.
void ReduceNhrLoop(const ScheduleParams& p, Builder& b)
{
    const uint32_t n = p.nRanks, me = p.rank;
    const bool isRoot = me == p.root;
    auto slice = [&](uint32_t i) { return CeilSlice(p.count, n, i); };
    // every rank reserves the working area in its staging (the root does not use it), so that all ranks cut the
    // same pieces
    const uint64_t workElems = AlignUp(p.count, std::max<uint64_t>(1, kAlignBytes / p.elemSize));
    auto work = [&](uint64_t off) { return isRoot ? Out(off) : Scr(off); };
    const uint64_t kSlots = 2;
    const uint64_t maxSlices = (n + 1) / 2;
    const uint64_t widest = slice(0).len;
    ScheduleParams pp = p;
    if (pp.scratchCapBytes != 0) pp.scratchCapBytes -= std::min(pp.scratchCapBytes, workElems * p.elemSize);
    const uint64_t pe = PieceElems(pp, widest, kSlots * maxSlices);
    const uint64_t np = std::max<uint64_t>(1, CeilDiv(widest, pe));
    auto slot = [&](uint64_t unit, size_t i) { return Scr(workElems + ((unit % kSlots) * maxSlices + i) * pe); };
    b.Copy(work(0), In(0), p.count);  // PreCopy (reduce_nhr.cc:140-162)
    uint64_t unit = 0;
    for (const NhrStep& st : NhrSteps(n, me, false)) {
        for (uint64_t t = 0; t < np; ++t, ++unit) {
            for (size_t i = 0; i < st.tx.size(); ++i) {
                Span s = Piece(slice(st.tx[i]), pe, t);
                b.Send(st.to, work(s.begin), s.len);
            }
            for (size_t i = 0; i < st.rx.size(); ++i) b.Recv(st.from, slot(unit, i), Piece(slice(st.rx[i]), pe, t).len);
            b.EndGroup();
            for (size_t i = 0; i < st.rx.size(); ++i) {
                Span s = Piece(slice(st.rx[i]), pe, t);
                b.Reduce(work(s.begin), {work(s.begin), slot(unit, i)}, s.len);
            }
        }
    }
    for (const NhrStep& st : NhrSteps(n, me, true)) {
        for (uint64_t t = 0; t < np; ++t) {
            for (size_t i = 0; i < st.tx.size(); ++i) {
                Span s = Piece(slice(st.tx[i]), pe, t);
                b.Send(st.to, work(s.begin), s.len);
            }
            for (size_t i = 0; i < st.rx.size(); ++i) {
                Span s = Piece(slice(st.rx[i]), pe, t);
                b.Recv(st.from, work(s.begin), s.len);
            }
            b.EndGroup();
        }
    }
}

void ReduceNhr(const ScheduleParams& p, Builder& b)
{
    ForEachRefLoop(p, b, RefLoopElems(p, kUbMaxDataSize, 1), [&](const ScheduleParams& lp) { ReduceNhrLoop(lp, b); });
}

// ------------------------------------------------------------------------------------------- AllGather

// Mesh: own block copied locally, every piece of the input sent to every peer in one group
// (the all-gather half of ins_temp_all_reduce_mesh_1D_two_shot.cc:340-432 as an operator).
void AllGatherMesh(const ScheduleParams& p, Builder& b)
{
    const uint32_t n = p.nRanks, me = p.rank;
    const uint64_t sc = p.count;
    const uint64_t pe = PieceElems(p, sc, 0);
    const uint64_t np = std::max<uint64_t>(1, CeilDiv(sc, pe));
    b.Copy(Out(uint64_t(me) * sc), In(0), sc);
    for (uint64_t t = 0; t < np; ++t) {
        Span s = Piece({0, sc}, pe, t);
        for (uint32_t q : PeerOrder(n, me)) {
            b.Send(q, In(s.begin), s.len);
            b.Recv(q, Out(uint64_t(q) * sc + s.begin), s.len);
        }
        b.EndGroup();
    }
}

// All-gather over R rings: part k of every block travels around ring k; step s forwards block cycle[v-s] to v+1 and
// receives block cycle[v-s-1] from v-1.
void AllGatherRing(const ScheduleParams& p, Builder& b)
{
    const uint32_t n = p.nRanks, me = p.rank;
    const uint64_t sc = p.count;
    const uint64_t alignElems = std::max<uint64_t>(1, kAlignBytes / p.elemSize);
    const std::vector<RingView> rings = Rings(n, me, sc * n * p.elemSize);
    const uint32_t R = static_cast<uint32_t>(rings.size());
    const uint64_t maxPart = RingPart(sc, R, 0, alignElems).len;
    const uint64_t pe = PieceElems(p, maxPart, 0);
    const uint64_t np = std::max<uint64_t>(1, CeilDiv(maxPart, pe));
    b.Copy(Out(uint64_t(me) * sc), In(0), sc);
    for (uint32_t s = 0; s + 1 < n; ++s) {
        for (uint64_t t = 0; t < np; ++t) {
            for (uint32_t k = 0; k < R; ++k) {
                const RingView& r = rings[k];
                const uint32_t bs = r.At(int64_t(r.pos) - s);
                const uint32_t br = r.At(int64_t(r.pos) - s - 1);
                const Span piece = Piece(RingPart(sc, R, k, alignElems), pe, t);
                b.Send(r.Next(), s == 0 ? In(piece.begin) : Out(uint64_t(bs) * sc + piece.begin), piece.len);
                b.Recv(r.Prev(), Out(uint64_t(br) * sc + piece.begin), piece.len);
            }
            b.EndGroup();
        }
    }
}

bool IsPow2(uint32_t n) { return n != 0 && (n & (n - 1)) == 0; }

}  // namespace

int32_t SelectAlgo(int32_t opType, uint32_t nRanks, uint64_t bytes, bool special)
{
    // DEFAULT_RANK_SIZE = 8.0 (auto_selector_base.h:28): AllReduce ratio 8/n/n, ReduceScatter (8/n)^2, in double
    const double n = nRanks == 0 ? 8.0 : double(nRanks);
    switch (opType) {
        case HCCL_AMD_OP_ALLREDUCE:
            if (bytes <= kOneShotMaxBytes) return HCCL_AMD_ALGO_MESH_ONESHOT;
            if (!special && double(bytes) * (8.0 / n / n) > double(32ull << 20)) return HCCL_AMD_ALGO_MESH_CHUNK;
            return HCCL_AMD_ALGO_MESH_TWOSHOT;
        case HCCL_AMD_OP_REDUCE_SCATTER:
            if (!special && double(bytes) * (8.0 / n) * (8.0 / n) > double(16ull << 20)) {
                return HCCL_AMD_ALGO_MESH_CHUNK;
            }
            return HCCL_AMD_ALGO_MESH_ONESHOT;
        case HCCL_AMD_OP_REDUCE:
            return bytes < kOneShotMaxBytes ? HCCL_AMD_ALGO_MESH_ONESHOT : HCCL_AMD_ALGO_MESH_TWOSHOT;
        case HCCL_AMD_OP_ALLGATHER: return HCCL_AMD_ALGO_MESH_ONESHOT;
        default: return HCCL_AMD_ALGO_AUTO;
    }
}

int BuildSchedule(const ScheduleParams& p, Schedule* out)
{
    if (p.nRanks == 0 || p.rank >= p.nRanks || p.elemSize == 0 || p.nRanks > HCCL_AMD_IR_MAX_SRC) {
        return HCCL_E_PARA;
    }
    if (p.opType == HCCL_AMD_OP_REDUCE && p.root >= p.nRanks) return HCCL_E_PARA;
    if (p.opType == HCCL_AMD_OP_REDUCE_SCATTER_V) {
        if (p.counts.size() != p.nRanks || p.displs.size() != p.nRanks) return HCCL_E_PARA;
        Builder bv;
        if (p.nRanks == 1) {
            bv.Copy(Out(0), In(p.displs[0]), p.counts[0]);
        } else {
            ReduceScatterVMesh(p, bv);  // the only AICPU template (reduce_scatter_v_auto_selector.cc:180-197)
        }
        out->ops = std::move(bv.ops);
        out->algo = HCCL_AMD_ALGO_MESH_ONESHOT;
        out->scratchElems = bv.scratchHigh;
        return HCCL_SUCCESS;
    }
    Builder b;
    int32_t algo = p.algo;
    uint64_t bytes = p.count * p.elemSize;
    if (algo == HCCL_AMD_ALGO_AUTO) algo = SelectAlgo(p.opType, p.nRanks, bytes, p.special);
    // The one-sided IPC collectives run as one kernel per executor loop, not as IR; their IR twins (same orders, same
    // bits) are the two-shot AllReduce / Reduce and the mesh ReduceScatter, which also run when the IPC path cannot.
    if (algo == HCCL_AMD_ALGO_IPC_TWOSHOT) algo = HCCL_AMD_ALGO_MESH_TWOSHOT;
    if (algo == HCCL_AMD_ALGO_IPC) algo = SelectAlgo(p.opType, p.nRanks, bytes, p.special);
    if (p.nRanks == 1) {
        // SingleRankProc (op_common.cc:3042-3098): a copy when the buffers differ.
        b.Copy(Out(0), In(0), p.count);
        out->ops = std::move(b.ops);
        out->algo = algo;
        out->scratchElems = 0;
        return HCCL_SUCCESS;
    }
    switch (p.opType) {
        case HCCL_AMD_OP_ALLREDUCE:
            if (algo == HCCL_AMD_ALGO_RHD && !IsPow2(p.nRanks)) algo = HCCL_AMD_ALGO_RING;
            switch (algo) {
                case HCCL_AMD_ALGO_MESH_ONESHOT: AllReduceOneShot(p, b); break;
                case HCCL_AMD_ALGO_MESH_TWOSHOT: AllReduceTwoShot(p, b); break;
                case HCCL_AMD_ALGO_RING: AllReduceRing(p, b); break;
                case HCCL_AMD_ALGO_RHD: AllReduceRhd(p, b); break;
                case HCCL_AMD_ALGO_NHR: AllReduceNhr(p, b); break;
                case HCCL_AMD_ALGO_ORDER_PRESERVED: AllReduceTree(p, b); break;
                case HCCL_AMD_ALGO_MESH_CHUNK: AllReduceMeshChunk(p, b); break;
                default: return HCCL_E_PARA;
            }
            break;
        case HCCL_AMD_OP_REDUCE_SCATTER:
            if (algo == HCCL_AMD_ALGO_MESH_TWOSHOT || algo == HCCL_AMD_ALGO_RHD) algo = HCCL_AMD_ALGO_MESH_ONESHOT;
            switch (algo) {
                case HCCL_AMD_ALGO_MESH_ONESHOT: ReduceScatterMesh(p, b); break;
                case HCCL_AMD_ALGO_NHR: ReduceScatterNhr(p, b); break;
                case HCCL_AMD_ALGO_RING: ReduceScatterRing(p, b); break;
                case HCCL_AMD_ALGO_ORDER_PRESERVED: ReduceScatterTree(p, b); break;
                case HCCL_AMD_ALGO_MESH_CHUNK: ReduceScatterMeshChunk(p, b); break;
                default: return HCCL_E_PARA;
            }
            break;
        case HCCL_AMD_OP_REDUCE:
            if (algo == HCCL_AMD_ALGO_RING || algo == HCCL_AMD_ALGO_RHD || algo == HCCL_AMD_ALGO_ORDER_PRESERVED ||
                algo == HCCL_AMD_ALGO_MESH_CHUNK) {
                algo = HCCL_AMD_ALGO_MESH_TWOSHOT;
            }
            switch (algo) {
                case HCCL_AMD_ALGO_MESH_ONESHOT: ReduceOneShot(p, b); break;
                case HCCL_AMD_ALGO_MESH_TWOSHOT: ReduceTwoShot(p, b); break;
                case HCCL_AMD_ALGO_NHR: ReduceNhr(p, b); break;
                default: return HCCL_E_PARA;
            }
            break;
        case HCCL_AMD_OP_ALLGATHER:
            if (algo != HCCL_AMD_ALGO_RING) algo = HCCL_AMD_ALGO_MESH_ONESHOT;
            if (algo == HCCL_AMD_ALGO_RING) {
                AllGatherRing(p, b);
            } else {
                AllGatherMesh(p, b);
            }
            break;
        default: return HCCL_E_PARA;
    }
    out->ops = std::move(b.ops);
    out->algo = algo;
    out->scratchElems = b.scratchHigh;
    return HCCL_SUCCESS;
}

}  // namespace hccl_amd
