// user_coll.cpp — host-evaluated reductions (user MPI_Op, x87 builtin ops; see user_coll.h).
//
// Data path.  Operands travel packed: each rank packs its operand on the device (the strided
// / run-table pack kernels; a host operand is packed on the host and uploaded) and each rank
// receives, device to device, only the packed element ranges it evaluates: an all-to-all of
// ranges over the point-to-point channels where the work is split by ranges (below), the whole
// operands (an allgather) where every rank evaluates every element.  The host then fetches only
// the element slices it evaluates, unpacks them into the type's layout — the user function is called on the derived
// type's layout, as the reference calls it on (char *)buf + disp * extent — runs the plan's
// programs (one uop(in, inout) call per program step and element block, the calls the
// reference's algorithm makes), packs the result's type-map bytes and returns them to the
// device, where one unpack writes the type map of recvbuf.  Gap bytes of recvbuf are never
// written (MPIR_Localcopy / Segment_unpack semantics, helper_fns.h:62-250).
//
// Work split.  Where every rank's program for an element is the same, every rank ends with the
// same bits and nobody needs to evaluate an element twice: the ring (chunk c is reduced by rank
// c and allgathered, allreduce_osu.c:3925-4005), the shmem / tree / two-level orders (reduced at
// local rank 0 and broadcast) and MPI_Reduce (only the root's result counts).  Those elements
// are split in n ranges, rank r evaluates range r (in the ring: its own chunk, as in the
// reference) and the packed results are allgathered, so each rank makes uop calls over (n-1)/n
// of the operand instead of n-1 whole operands, and receives (n-1)/n of one operand's bytes
// (the reference's ring moves 2(n-1)/n of it per rank, allreduce_osu.c:3925-4005: the reduce-
// scatter half here, the results' allgather the other).  MPI_Reduce gathers the results at the
// root only; MPI_Reduce_scatter moves each rank only its own block of every operand.  Where the
// programs differ between ranks
// (recursive doubling, :360-630: each rank's own bracketing) every rank evaluates its own
// result over every element, from the packed operands.
//
// Several nodes.  The operands travel the same way over the whole job (the packed allgather
// crosses the leaders' links) and the schedule is the one the device path restates there
// (runtime/coll.cpp mn_host_schedule): flat schedules are evaluated as above over the job's ranks;
// a two-level schedule is evaluated in its two stages — each node's partial at its leader (the
// node step's programs over that node's operands), then the leaders' programs over the partials.
#include "user_coll.h"

#include <hip/hip_runtime.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <chrono>
#include <vector>

#include "../../../include/mv2h.h"
#include "../common.h"
#include "../runtime/orders.h"
#include "../runtime/pvars.h"
#include "../runtime/world.h"
#include "datatype.h"

namespace mv2 {

void HostBuf::resize(size_t n) {
    static char *buf[HS_COUNT];
    static size_t cap[HS_COUNT];
    static bool pinned[HS_COUNT];
    if (n > cap[slot_]) {
        if (buf[slot_]) {
            if (pinned[slot_]) (void)hipHostFree(buf[slot_]);
            else free(buf[slot_]);
        }
        const size_t want = std::max(n, 2 * cap[slot_]);
        void *q = nullptr;
        pinned[slot_] = hipHostMalloc(&q, want, hipHostMallocDefault) == hipSuccess;
        if (!pinned[slot_]) {
            (void)hipGetLastError();
            q = malloc(want);  // no GPU (host-buffer x87 calls): plain memory
        }
        buf[slot_] = (char *)q;
        cap[slot_] = q ? want : 0;
    }
    p_ = buf[slot_];
    n_ = n;
}

namespace {

// device scratch kept between calls, grown on demand
enum DevSlot { DS_MINE, DS_ALL, DS_RES_MINE, DS_RES_ALL, DS_REM, DS_SPAN, DS_COUNT };
char *dev_scratch(int slot, size_t bytes) {
    static void *p[DS_COUNT];
    static size_t cap[DS_COUNT];
    if (bytes == 0) bytes = 1;
    if (bytes > cap[slot]) {
        // an abandoned collective receive may still be arriving into the old block (DS_ALL /
        // DS_RES_ALL are receive areas): then it is left allocated rather than freed under it
        if (p[slot] && !coll_context_poisoned()) mv2h_free(p[slot]);
        p[slot] = nullptr;
        cap[slot] = 0;
        ++world().call_allocs;
        if (mv2h_malloc(&p[slot], bytes)) return (char *)(p[slot] = nullptr);
        cap[slot] = bytes;
    }
    return (char *)p[slot];
}

// the ranks a reduction runs over: the node's, or every rank of a job on several nodes
struct Job {
    int n, me;
    bool multi;
};
Job job() {
    const World &w = world();
    return w.nnodes > 1 ? Job{w.gsize, w.grank, true} : Job{w.size, w.rank, false};
}

// Phase accounting of a host-evaluated call (World::uop_ns, mv2h_get_info "uop_*_us"): mark(p)
// charges the time since the previous mark to phase p.
enum UopPhase { UP_STAGE, UP_FETCH, UP_EVAL, UP_DELIVER };

// Where a derived layout's gaps are handled: on the device (spans cross PCIe, gaps included) or
// on the host (packed bytes cross PCIe, the host's block loop writes the spans).  A sparse span
// costs the device route its gap bytes on the link, the host route a read-for-ownership pass over
// the span; the link is the GPU's, shared by the ranks on it, the host loop is each rank's own
// core.  Measured on the configs[4] vector (half gaps): the device route wins with the link to
// itself or shared by 2 (4.4 -> 3.6 ms per call), the host route with 8 ranks on one link
// (7.5 -> 10 ms); the crossover of the two costs is at a few ranks per link.
bool layout_on_device() { return world().nshare <= 4; }
struct PhaseClock {
    std::chrono::steady_clock::time_point t = std::chrono::steady_clock::now();
    void mark(int phase) {
        const auto now = std::chrono::steady_clock::now();
        world().uop_ns[phase] += (uint64_t)std::chrono::duration_cast<std::chrono::nanoseconds>(now - t).count();
        t = now;
    }
};

struct Typed {
    MPI_Datatype dt;
    long tsize, extent;
    bool contig;  // the packed layout is the type's layout
};

Typed typed(MPI_Datatype dt) {
    Typed t{dt, dtype_size(dt), dtype_extent(dt), false};
    t.contig = dtype_is_contiguous(dt) && t.tsize == t.extent;
    return t;
}

// every rank's operand, packed, on the device, for elements [lo, hi): rank j's element e at
// all + j * stride + (e - lo) * tsize
struct Operands {
    Typed t;
    int n;
    size_t P;  // one whole packed operand
    const char *all;
    size_t stride;
    long lo, hi;
};

constexpr int kTagRanges = kCollTagBase - 4;  // the library's collective context (runtime/world.h)

// this rank's operand packed on the device (DS_MINE)
int pack_mine(const void *src, int count, const Typed &t, char **out) {
    const size_t P = (size_t)count * (size_t)t.tsize;
    char *mine = dev_scratch(DS_MINE, P);
    if (!mine) return MPI_ERR_NO_MEM;
    int rc;
    if (mv2h_is_device_ptr(src)) {
        rc = dtype_pack(src, count, t.dt, mine);
    } else {
        HostBuf h(HS_PACKED);
        h.resize(P + 1);
        if (!h.data()) return MPI_ERR_NO_MEM;
        rc = dtype_pack(src, count, t.dt, h.data());
        if (!rc && mv2h_memcpy_htod(mine, h.data(), P)) rc = MPI_ERR_OTHER;
    }
    *out = mine;
    return rc;
}

// every rank's whole packed operand on every rank (the device allgather)
int gather_whole(const char *mine, int count, const Typed &t, int slot, Operands &o) {
    o.t = t;
    o.n = job().n;
    o.P = (size_t)count * (size_t)t.tsize;
    char *all = dev_scratch(slot, o.P * (size_t)o.n);
    if (!all) return MPI_ERR_NO_MEM;
    o.all = all;
    o.stride = o.P;
    o.lo = 0;
    o.hi = count;
    world().uop_in_bytes = o.P * (size_t)(o.n - 1);
    world().uop_area_bytes = o.P * (size_t)o.n;
    if (o.n == 1) return mv2h_memcpy_dtod(all, mine, o.P) ? MPI_ERR_OTHER : 0;
    return mv2h_allgather(mine, all, o.P, nullptr);
}

// the point-to-point channels reach every rank of the job (every node's ranks up to the rank mesh)
bool channels_reach_all() {
    const World &w = world();
    return w.nnodes == 1 || w.gsize <= kMeshMaxRanks;
}

// Elements [lo[me], hi[me]) of every rank's packed operand onto this rank (rank j's at
// all + j * stride): an all-to-all of ranges over the point-to-point channels, each rank sent
// only the range it evaluates.  Beyond the channels' reach: the whole operands, windowed.
int exchange_ranges(const char *mine, int count, const Typed &t, const std::vector<long> &lo,
                    const std::vector<long> &hi, Operands &o) {
    const Job J = job();
    const int n = J.n, me = J.me;
    if (!channels_reach_all()) {
        const int rc = gather_whole(mine, count, t, DS_ALL, o);
        if (rc) return rc;
        o.all += (size_t)lo[me] * (size_t)t.tsize;
        o.lo = lo[me];
        o.hi = hi[me];
        return 0;
    }
    const size_t ts = (size_t)t.tsize, mb = (size_t)(hi[me] - lo[me]) * ts;
    char *all = dev_scratch(DS_ALL, mb * (size_t)n);
    if (!all) return MPI_ERR_NO_MEM;
    o.t = t;
    o.n = n;
    o.P = (size_t)count * ts;
    o.all = all;
    o.stride = mb;
    o.lo = lo[me];
    o.hi = hi[me];
    world().uop_in_bytes = mb * (size_t)(n - 1);
    world().uop_area_bytes = mb * (size_t)n;
    std::vector<unsigned long long> reqs;
    reqs.reserve(2 * (size_t)n);
    int rc = 0;
    for (int j = 0; j < n && !rc; ++j) {
        if (j == me || !mb) continue;
        unsigned long long q = 0;
        if (!(rc = p2p_irecv(all + (size_t)j * mb, mb, j, kTagRanges, &q))) reqs.push_back(q);
    }
    for (int j = 0; j < n && !rc; ++j) {
        const size_t jb = (size_t)(hi[j] - lo[j]) * ts;
        if (j == me || !jb) continue;
        unsigned long long q = 0;
        if (!(rc = p2p_isend(mine + (size_t)lo[j] * ts, jb, j, kTagRanges, &q))) reqs.push_back(q);
    }
    if (!rc && mb && mv2h_memcpy_dtod(all + (size_t)me * mb, mine + (size_t)lo[me] * ts, mb)) rc = MPI_ERR_OTHER;
    for (unsigned long long q : reqs) {
        if (rc) {
            p2p_abandon(q);
            continue;
        }
        if ((rc = mv2h_p2p_wait(q, nullptr, nullptr, nullptr))) p2p_abandon(q);
    }
    return rc ? MPI_ERR_OTHER : 0;
}

// the whole packed operands on every rank (every element evaluated by every rank)
int stage_operands(const void *src, int count, const Typed &t, Operands &o) {
    char *mine = nullptr;
    const int rc = pack_mine(src, count, t, &mine);
    return rc ? rc : gather_whole(mine, count, t, DS_ALL, o);
}

// Elements [b, e) of every rank's operand in the type's layout (element b at offset 0),
// operand j at W + j * rspan
int fetch(const Operands &o, long b, long e, HostBuf &W, long &rspan) {
    const Typed &t = o.t;
    const int cnt = (int)(e - b);
    if (b < o.lo || e > o.hi) return MPI_ERR_INTERN;  // outside what this rank received
    rspan = dtype_span(t.dt, cnt);
    const size_t rb = (size_t)cnt * (size_t)t.tsize;
    W.resize((size_t)rspan * (size_t)o.n + 1);
    if (!W.data()) return MPI_ERR_NO_MEM;
    if (!cnt) return 0;
    const char *src = o.all + (size_t)(b - o.lo) * (size_t)t.tsize;
    if (t.contig)  // the slices land in place: one strided copy
        return hipMemcpy2D(W.data(), (size_t)rspan, src, o.stride, rb, (size_t)o.n, hipMemcpyDeviceToHost) == hipSuccess
                   ? 0 : MPI_ERR_OTHER;
    // a derived layout: unpacked on the device (one kernel per operand), then one copy of the
    // n spans — the host's own block loop over a sparse layout reads-for-ownership every line
    // it half-writes, several times slower than moving the gaps over PCIe (r04r: 3.7 ms of a
    // 4.4 ms call at 2 ranks)
    if (char *sp = layout_on_device() ? dev_scratch(DS_SPAN, (size_t)rspan * (size_t)o.n) : nullptr) {
        for (int j = 0; j < o.n; ++j) {
            const int rc = dtype_unpack(src + (size_t)j * o.stride, cnt, t.dt, sp + (size_t)j * (size_t)rspan);
            if (rc) return rc;
        }
        return mv2h_memcpy_dtoh(W.data(), sp, (size_t)rspan * (size_t)o.n) ? MPI_ERR_OTHER : 0;
    }
    HostBuf pk(HS_PACKED);
    pk.resize(rb * (size_t)o.n + 1);
    if (!pk.data()) return MPI_ERR_NO_MEM;
    if (hipMemcpy2D(pk.data(), rb, src, o.stride, rb, (size_t)o.n, hipMemcpyDeviceToHost) != hipSuccess) return MPI_ERR_OTHER;
    for (int j = 0; j < o.n; ++j) {
        const int rc = dtype_unpack(pk.data() + (size_t)j * rb, cnt, t.dt, W.data() + (size_t)j * (size_t)rspan);
        if (rc) return rc;
    }
    return 0;
}

// Run ps over elements [b, e) held in W (element b at offset 0 of each operand, rspan bytes
// apart); program blocks count from element `pbase`.  Step s is fn(in = w[src], inout = w[dst]).
// The result's type-map bytes are packed into out (element b first).
int eval_range(const ProgSet &ps, long pbase, char *W, long rspan, long b, long e, const Typed &t,
               MPI_User_function *fn, char *out) {
    for (long x = b; x < e;) {
        int k = 0;
        long xe = e;
        if (ps.nprog > 1) {
            k = (int)std::min<long>((x - pbase) / (long)ps.blk, ps.nprog - 1);
            if (k < ps.nprog - 1) xe = std::min<long>(e, pbase + (long)(k + 1) * (long)ps.blk);
        }
        const Prog &p = ps.p[k];
        const size_t off = (size_t)(x - b) * (size_t)t.extent;
        for (int s = 0; s < p.nsteps; ++s) {
            int cnt = (int)(xe - x);
            MPI_Datatype d = t.dt;
            fn(W + (size_t)p.src[s] * rspan + off, W + (size_t)p.dst[s] * rspan + off, &cnt, &d);
        }
        const int rc = dtype_pack(W + (size_t)p.res * rspan + off, (int)(xe - x), t.dt, out + (size_t)(x - b) * t.tsize);
        if (rc) return rc;
        x = xe;
    }
    return 0;
}

int eval_into(const ProgSet &ps, long pbase, char *W, long rspan, long b, long e, const Typed &t,
              MPI_User_function *fn, char *dst);

// eval_range with the packed result on the device at dev_out: a derived layout's result goes up
// in the type's layout and is packed there (the host's pack loop is the slow part, see fetch)
int eval_to_device(const ProgSet &ps, long pbase, char *W, long rspan, long b, long e, const Typed &t,
                   MPI_User_function *fn, char *dev_out) {
    const size_t pb = (size_t)(e - b) * (size_t)t.tsize;
    if (e <= b) return 0;
    int rc;
    if (!t.contig && layout_on_device()) {
        const long span = dtype_span(t.dt, (int)(e - b));
        char *sp = dev_scratch(DS_SPAN, (size_t)span);
        if (sp && ps.nprog == 1) {  // one program: its steps in place, the result register goes up as it is
            const Prog &p = ps.p[0];
            for (int s = 0; s < p.nsteps; ++s) {
                int cnt = (int)(e - b);
                MPI_Datatype d = t.dt;
                fn(W + (size_t)p.src[s] * rspan, W + (size_t)p.dst[s] * rspan, &cnt, &d);
            }
            if (mv2h_memcpy_htod(sp, W + (size_t)p.res * rspan, (size_t)span)) return MPI_ERR_OTHER;
            return dtype_pack(sp, (int)(e - b), t.dt, dev_out);
        }
        HostBuf R(HS_RESULT);
        R.resize((size_t)span + 1);
        if (R.data() && sp) {
            if ((rc = eval_into(ps, pbase, W, rspan, b, e, t, fn, R.data()))) return rc;
            if (mv2h_memcpy_htod(sp, R.data(), (size_t)span)) return MPI_ERR_OTHER;
            return dtype_pack(sp, (int)(e - b), t.dt, dev_out);
        }
    }
    HostBuf R(HS_RESULT);
    R.resize(pb + 1);
    if (!R.data()) return MPI_ERR_NO_MEM;
    if ((rc = eval_range(ps, pbase, W, rspan, b, e, t, fn, R.data()))) return rc;
    return mv2h_memcpy_htod(dev_out, R.data(), pb) ? MPI_ERR_OTHER : 0;
}

bool same_progs(const ProgSet &a, const ProgSet &b) {
    if (a.nprog != b.nprog || (a.nprog > 1 && a.blk != b.blk)) return false;
    for (int k = 0; k < a.nprog; ++k) {
        const Prog &p = a.p[k], &q = b.p[k];
        if (p.nsteps != q.nsteps || p.res != q.res) return false;
        for (int s = 0; s < p.nsteps; ++s)
            if (p.dst[s] != q.dst[s] || p.src[s] != q.src[s]) return false;
    }
    return true;
}

// Elements [0, U) have the same programs on every rank (uni) and are split over the ranks;
// [U, count) are this rank's own (own, program blocks counted from own_base)
struct Split {
    const ProgSet *uni;
    long U;
    const ProgSet *own;
    long own_base;
};

// The operands a split needs, staged: the uniform part [0, U) by ranges (rank r gets range r of
// every operand, ou), the own part [U, count) whole on every rank (oo; an allgather of those
// elements only).  U = 0: every rank's whole operand (recursive doubling: each rank's own tree).
int stage_split(const void *src, int count, const Typed &t, const Split &sp, Operands &ou, Operands &oo) {
    char *mine = nullptr;
    int rc = pack_mine(src, count, t, &mine);
    if (rc) return rc;
    if (sp.U == 0) return gather_whole(mine, count, t, DS_ALL, oo);
    const int n = job().n;
    const long chunk = (sp.U + n - 1) / n;
    std::vector<long> lo((size_t)n), hi((size_t)n);
    for (int j = 0; j < n; ++j) {
        lo[j] = std::min<long>(sp.U, (long)j * chunk);
        hi[j] = std::min<long>(sp.U, lo[j] + chunk);
    }
    if ((rc = exchange_ranges(mine, count, t, lo, hi, ou))) return rc;
    if (sp.U < count) {  // the own part: those elements of every operand
        const size_t rb = (size_t)(count - sp.U) * (size_t)t.tsize;
        char *rem = dev_scratch(DS_REM, rb * (size_t)n);
        if (!rem) return MPI_ERR_NO_MEM;
        if ((rc = mv2h_allgather(mine + (size_t)sp.U * (size_t)t.tsize, rem, rb, nullptr))) return rc;
        oo = Operands{t, n, (size_t)count * (size_t)t.tsize, rem, rb, sp.U, count};
    }
    return 0;
}

// Every rank's range of results (packed; range j of `chunk` elements, the last ones short or empty)
// into res_all at j * chunk: allgathered (root < 0), or gathered at the root over the point-to-point
// channels (MPI_Reduce: only the root's result counts)
int collect_results(const char *res_mine, char *res_all, long U, long chunk, size_t tsize, int root) {
    const Job J = job();
    const int n = J.n, me = J.me;
    const size_t cb = (size_t)chunk * tsize;
    if (root < 0 || !channels_reach_all()) return mv2h_allgather(res_mine, res_all, cb, nullptr);
    auto bytes_of = [&](int j) { return (size_t)(std::min<long>(U, (long)(j + 1) * chunk) - std::min<long>(U, (long)j * chunk)) * tsize; };
    int rc = 0;
    unsigned long long q = 0;
    if (me != root) {
        if (!bytes_of(me)) return 0;
        if ((rc = p2p_isend(res_mine, bytes_of(me), root, kTagRanges, &q))) return MPI_ERR_OTHER;
        if ((rc = mv2h_p2p_wait(q, nullptr, nullptr, nullptr))) p2p_abandon(q);
        return rc ? MPI_ERR_OTHER : 0;
    }
    std::vector<unsigned long long> reqs;
    for (int j = 0; j < n && !rc; ++j) {
        if (j == me || !bytes_of(j)) continue;
        if (!(rc = p2p_irecv(res_all + (size_t)j * cb, bytes_of(j), j, kTagRanges, &q))) reqs.push_back(q);
    }
    if (!rc && bytes_of(me) && mv2h_memcpy_dtod(res_all + (size_t)me * cb, res_mine, bytes_of(me))) rc = MPI_ERR_OTHER;
    for (unsigned long long r : reqs) {
        if (rc) {
            p2p_abandon(r);
            continue;
        }
        if ((rc = mv2h_p2p_wait(r, nullptr, nullptr, nullptr))) p2p_abandon(r);
    }
    return rc ? MPI_ERR_OTHER : 0;
}

// root < 0: every rank delivers the result; root >= 0: the root only
int run_split(const void *src, int count, const Typed &t, const Split &sp, MPI_User_function *fn, void *recvbuf,
              int root) {
    const int n = job().n, me = job().me;
    const bool deliver = root < 0 || me == root;
    PhaseClock pc;
    Operands ou{}, oo{};
    int rc = stage_split(src, count, t, sp, ou, oo);
    if (rc) return rc;
    pc.mark(UP_STAGE);
    const long chunk = sp.U ? (sp.U + n - 1) / n : 0;
    const long mb = std::min<long>(sp.U, (long)me * chunk), me_e = std::min<long>(sp.U, mb + chunk);
    char *res_all = dev_scratch(DS_RES_ALL, (size_t)std::max<long>((long)n * chunk, count) * (size_t)t.tsize);
    if (!res_all) return MPI_ERR_NO_MEM;
    HostBuf W(HS_OPERANDS), R(HS_RESULT);
    long rspan = 0;
    if (sp.U > 0) {
        const size_t cb = (size_t)chunk * (size_t)t.tsize;
        char *res_mine = dev_scratch(DS_RES_MINE, cb);
        R.resize(cb + 1);
        if (!res_mine || !R.data()) return MPI_ERR_NO_MEM;
        if (me_e > mb) {
            if ((rc = fetch(ou, mb, me_e, W, rspan))) return rc;
            pc.mark(UP_FETCH);
            if ((rc = eval_to_device(*sp.uni, 0, W.data(), rspan, mb, me_e, t, fn, res_mine))) return rc;
            pc.mark(UP_EVAL);
        }
        // a short (or empty) last range leaves its padding at or after element U, where the
        // own part below (or nothing) lands
        if ((rc = collect_results(res_mine, res_all, sp.U, chunk, (size_t)t.tsize, root))) return rc;
        pc.mark(UP_DELIVER);
    }
    if (sp.U < count && deliver) {
        if ((rc = fetch(oo, sp.U, count, W, rspan))) return rc;
        pc.mark(UP_FETCH);
        if ((rc = eval_to_device(*sp.own, sp.own_base, W.data(), rspan, sp.U, count, t, fn,
                                 res_all + (size_t)sp.U * t.tsize)))
            return rc;
        pc.mark(UP_EVAL);
    }
    rc = deliver ? dtype_unpack(res_all, count, t.dt, recvbuf) : 0;
    pc.mark(UP_DELIVER);
    return rc;
}

// Run ps over elements [b, e) of the nreg operands at W (rspan bytes apart, element b at offset 0),
// program blocks counted from element pbase, and copy each element's result into dst (the type's
// layout, element b at offset 0)
int eval_into(const ProgSet &ps, long pbase, char *W, long rspan, long b, long e, const Typed &t,
              MPI_User_function *fn, char *dst) {
    for (long x = b; x < e;) {
        int k = 0;
        long xe = e;
        if (ps.nprog > 1) {
            k = (int)std::min<long>((x - pbase) / (long)ps.blk, ps.nprog - 1);
            if (k < ps.nprog - 1) xe = std::min<long>(e, pbase + (long)(k + 1) * (long)ps.blk);
        }
        const Prog &p = ps.p[k];
        const size_t off = (size_t)(x - b) * (size_t)t.extent;
        for (int s = 0; s < p.nsteps; ++s) {
            int cnt = (int)(xe - x);
            MPI_Datatype d = t.dt;
            fn(W + (size_t)p.src[s] * rspan + off, W + (size_t)p.dst[s] * rspan + off, &cnt, &d);
        }
        const long span = dtype_span(t.dt, (int)(xe - x));
        memcpy(dst + off, W + (size_t)p.res * rspan + off, (size_t)span);
        x = xe;
    }
    return 0;
}

// ---- more ranks (or leaders) than a program holds: the message schedules restated on the host ----
// W holds `n` operands in the type's layout, rspan bytes apart, cnt elements each; every function
// writes one rank's result (type layout, rspan bytes) to out and leaves W unchanged.
struct BigEval {
    const char *W;
    long rspan;
    int n, cnt;
    const Typed *t;
    MPI_User_function *fn;
    bool comm;
    std::vector<std::vector<char>> scratch;  // one operand-sized buffer per recursion level
    // MPIR_Reduce_redscat_gather_MV2's pre-step (reduce_osu.c:849-894: odd ranks below 2 * rem hand
    // their operand to rank - 1, the even ones keep their place) instead of the allreduce's
    bool redscat = false;
    char *level(int l) {
        if ((int)scratch.size() <= l) scratch.resize((size_t)l + 1);
        if (scratch[l].size() < (size_t)rspan + 1) scratch[l].resize((size_t)rspan + 1);
        return scratch[l].data();
    }
    void uop(const char *in, char *inout) {
        int c = cnt;
        MPI_Datatype d = t->dt;
        fn((void *)in, inout, &c, &d);
    }
    const char *x(int r) const { return W + (size_t)r * (size_t)rspan; }
    // one operand's cnt elements (a sub-range's span, not the stride: W may start mid-operand)
    void copy(char *dst, const char *src) const { memcpy(dst, src, (size_t)dtype_span(t->dt, cnt)); }

    int pof2() const {
        int p = 1;
        while (p * 2 <= n) p *= 2;
        return p;
    }
    int real(int q) const {
        const int rem = n - pof2();
        return q < rem ? q * 2 + (redscat ? 0 : 1) : q + rem;
    }
    // the non-power-of-two pre-step: newrank nr's starting value (an odd rank below 2 * rem has
    // reduced uop(tmp = x_{r-1}, recvbuf); redscat_gather: an even one uop(tmp = x_{r+1}, recvbuf))
    void base(int nr, char *out) {
        const int r = real(nr);
        copy(out, x(r));
        if (r < 2 * (n - pof2())) uop(x(redscat ? r + 1 : r - 1), out);
    }
    // MPIR_Allreduce_pt2pt_rd_MV2 (allreduce_osu.c:455-600; also pt2pt_rs for a user op, :802): the
    // value newrank nr holds after `lev` doubling steps
    void rd_value(int nr, int lev, char *out) {
        if (lev == 0) return base(nr, out);
        const int mask = 1 << (lev - 1), pr = nr ^ mask;
        char *other = level(lev);
        rd_value(nr, lev - 1, out);
        rd_value(pr, lev - 1, other);
        if (comm || real(pr) < real(nr)) {
            uop(other, out);  // uop(tmp_buf, recvbuf)
        } else {
            uop(out, other);  // uop(recvbuf, tmp_buf), then tmp_buf copied into recvbuf
            copy(out, other);
        }
    }
    // MPIR_Allreduce_pt2pt_rs_MV2's reduce-scatter + allgather (:852-1000; builtin ops, at least
    // pof2 elements): block i of pof2 (count / pof2 elements, the last the remainder) is reduced
    // at the newrank whose bits are i's reversed (each halving step keeps the lower half at the
    // lower newrank), along the same doubling steps as recursive doubling at that newrank, and
    // the allgather gives every rank every block
    void rs(char *out) {
        int pof2 = 1, lev = 0;
        while (pof2 * 2 <= n) pof2 *= 2, ++lev;
        const int whole = cnt;
        const long per = whole / pof2;
        for (int i = 0; i < pof2; ++i) {
            const long b = (long)i * per, c = i < pof2 - 1 ? per : whole - per * (pof2 - 1);
            int owner = 0;
            for (int j = 0; j < lev; ++j) owner = (owner << 1) | ((i >> j) & 1);
            BigEval sub{W + (size_t)b * (size_t)t->extent, rspan, n, (int)c, t, fn, comm, {}};
            sub.redscat = redscat;  // the block keeps redscat_gather's pre-step
            std::vector<char> part((size_t)rspan + 1);
            sub.rd_value(owner, lev, part.data());
            memcpy(out + (size_t)b * (size_t)t->extent, part.data(), (size_t)dtype_span(t->dt, (int)c));
        }
    }
    // rank me's recursive-doubling result
    void rd(int me, char *out) {
        int pof2 = 1, lev = 0;
        while (pof2 * 2 <= n) pof2 *= 2, ++lev;
        const int rem = n - pof2;
        // an even rank below 2 * rem takes rank + 1's result in the post-step
        const int nr = me < 2 * rem ? me / 2 : me - rem;
        rd_value(nr, lev, out);
    }
    // MPI_Reduce_scatter, this rank's block (W holds its elements of every operand; commutative
    // ops).  MPIR_Reduce_scatter_Rec_Halving_MV2 (red_scat_osu.c:428-780): the pre-step, then
    // halving steps with masks pof2/2, pof2/4, ... 1, each uop(tmp_recvbuf, tmp_results); newrank i
    // ends with new block i, which holds rank i's block (and, below 2 * rem, its even neighbour's)
    void rh_value(int nr, int k, int lev, char *out) {
        if (k == 0) return base(nr, out);
        const int mask = (1 << lev) >> k;
        char *other = level(k);
        rh_value(nr, k - 1, lev, out);
        rh_value(nr ^ mask, k - 1, lev, other);
        uop(other, out);
    }
    void rs_halving(int me, char *out) {
        int p = 1, lev = 0;
        while (p * 2 <= n) p *= 2, ++lev;
        const int rem = n - p;
        rh_value(me < 2 * rem ? me / 2 : me - rem, lev, lev, out);
    }
    // MPIR_Reduce_scatter_Pair_Wise_MV2 (:786-1020): own data, then uop(x_{me-i}, acc), i = 1 .. n-1
    void rs_pairwise(int me, char *out) {
        copy(out, x(me));
        for (int i = 1; i < n; ++i) uop(x((me - i + n) % n), out);
    }
    // MPIR_Reduce_scatter_ring (:1026-1180): the block starts at rank me + 1; each next rank
    // reduces the partial it receives into its own data, uop(tmp_recvbuf, tmp_sendbuf)
    void rs_ring(int me, char *out) {
        char *acc = level(0), *next = level(1);
        copy(acc, x((me + 1) % n));
        for (int j = 2; j <= n; ++j) {
            copy(next, x((me + j) % n));
            uop(acc, next);
            std::swap(acc, next);
        }
        copy(out, acc);
    }
    // MPIR_Reduce_binomial_MV2 (reduce_osu.c:577-663): relative rank rel's value once the masks
    // below m are done (a non-commutative op reduces towards rank 0, which forwards to the root)
    void bin_value(int rel, int m, int lroot, int l, char *out) {
        if (m == 1) {
            copy(out, x((rel + lroot) % n));
            return;
        }
        const int half = m / 2;
        bin_value(rel, half, lroot, l + 1, out);
        if ((rel | half) >= n) return;
        char *child = level(l);
        bin_value(rel | half, half, lroot, l + 1, child);
        if (comm) {
            uop(child, out);  // uop(tmp_buf, recvbuf)
        } else {
            uop(out, child);  // uop(recvbuf, tmp_buf), then tmp_buf copied into recvbuf
            copy(out, child);
        }
    }
    void binomial(int root, char *out) {
        int m = 1;
        while (m < n) m <<= 1;
        bin_value(0, m, comm ? root : 0, 0, out);
    }
    // MPIR_Reduce_knomial_MV2 (reduce_osu.c:1639-1837) to `root`: relative rank rel's value is its
    // own operand reduced with its children's values (MPIR_Reduce_knomial_trace :1568-1633), the
    // trace's last child first (request-index order), uop(tmp, recvbuf)
    void knom_value(int rel, int root, int k, int l, char *out) {
        copy(out, x((rel + root) % n));
        int mask = 1;
        while (mask < n && !(rel % (k * mask))) mask *= k;
        mask /= k;
        std::vector<int> kids;
        for (int m = mask; m > 0; m /= k)
            for (int j = 1; j < k; ++j)
                if (rel + m * j < n) kids.push_back(rel + m * j);
        char *child = level(l);
        for (size_t i = kids.size(); i-- > 0;) {
            knom_value(kids[i], root, k, l + 1, child);
            uop(child, out);
        }
    }
    void knomial(int root, int k, char *out) { knom_value(0, root, k < 2 ? 2 : k, 0, out); }
    // MPIR_Reduce_redscat_gather_MV2 (reduce_osu.c:718-1100): its reduce-scatter (the recursive
    // halving of pt2pt_rs after its own pre-step), the gather to the root
    void redscat_gather(char *out) {
        redscat = true;
        rs(out);
        redscat = false;
    }
    // an expression tree (orders.h ExprNode) over the n operands: node e's value into out
    void expr(const std::vector<ExprNode> &nodes, int e, int l, char *out) {
        const ExprNode &nd = nodes[(size_t)e];
        if (nd.leaf >= 0) {
            copy(out, x(nd.leaf));
            return;
        }
        expr(nodes, nd.a, l + 1, out);  // the inout operand
        char *in = level(l);
        expr(nodes, nd.b, l + 1, in);
        uop(in, out);
    }
    // MPIR_Allreduce_pt2pt_ring_MV2's chunk c (allreduce_osu.c:3916-3968): x_c, then uop(x_{c+j},
    // acc) for j = 1 .. n-1
    void ring_chunk(int c, char *out) {
        copy(out, x(c));
        for (int j = 1; j < n; ++j) uop(x((c + j) % n), out);
    }
};

// Big flat schedules over the job's operands (MnSched big, kind MN_FLAT); deliver: this rank
// takes the result (MPI_Reduce: the root only)
int run_big_flat(const Operands &o, int count, const MnSched &sc, const HostOp &op, void *recvbuf, bool deliver) {
    const Typed &t = o.t;
    const int n = o.n, me = job().me;
    char *res_all = dev_scratch(DS_RES_ALL, (size_t)count * (size_t)t.tsize);
    if (!res_all) return MPI_ERR_NO_MEM;
    HostBuf W(HS_OPERANDS), R(HS_RESULT);
    long rspan = 0;
    int rc = 0;
    auto eval = [&](long b, long e, auto &&body) -> int {
        if (e <= b) return 0;
        if ((rc = fetch(o, b, e, W, rspan))) return rc;
        BigEval ev{W.data(), rspan, n, (int)(e - b), &t, op.fn, op.opk != OPK_USER_NONCOMM, {}};
        std::vector<char> out((size_t)rspan + 1);
        body(ev, out.data());
        R.resize((size_t)(e - b) * (size_t)t.tsize + 1);
        if (!R.data()) return MPI_ERR_NO_MEM;
        return dtype_pack(out.data(), (int)(e - b), t.dt, R.data());
    };
    long U = 0;
    if (sc.forced == ALG_RING) {
        // rank r reduces ring chunk r (the reference's own split) and the chunks are allgathered
        U = sc.U;
        const long cc = U / n;
        const size_t cb = (size_t)cc * (size_t)t.tsize;
        char *res_mine = dev_scratch(DS_RES_MINE, cb);
        if (!res_mine) return MPI_ERR_NO_MEM;
        if ((rc = eval((long)me * cc, (long)(me + 1) * cc, [&](BigEval &ev, char *out) { ev.ring_chunk(me, out); })))
            return rc;
        if (cc && mv2h_memcpy_htod(res_mine, R.data(), cb)) return MPI_ERR_OTHER;
        if ((rc = mv2h_allgather(res_mine, res_all, cb, nullptr))) return rc;
    }
    // pt2pt_rs on [b, e): its reduce-scatter for a builtin op over at least pof2 elements, else
    // recursive doubling (:802)
    int pof2 = 1;
    while (pof2 * 2 <= n) pof2 *= 2;
    auto segment = [&](long b, long e, int algo) -> int {
        if (e <= b) return 0;
        const int r = eval(b, e, [&](BigEval &ev, char *out) {
            if (algo == ALG_BINOMIAL) ev.binomial(sc.root, out);
            else if (algo == ALG_KNOMIAL) ev.knomial(sc.root, sc.k, out);
            else if (algo == ALG_REDSCAT_GATHER) ev.redscat_gather(out);
            else if (algo == ALG_PT2PT_RS && op.opk == OPK_BUILTIN && e - b >= pof2) ev.rs(out);
            else ev.rd(me, out);
        });
        if (r) return r;
        return mv2h_memcpy_htod(res_all + (size_t)b * (size_t)t.tsize, R.data(), (size_t)(e - b) * (size_t)t.tsize)
                   ? MPI_ERR_OTHER : 0;
    };
    if ((sc.forced == ALG_BINOMIAL || sc.forced == ALG_KNOMIAL || sc.forced == ALG_REDSCAT_GATHER) && !deliver) return 0;
    if (sc.forced == ALG_RING) {
        rc = segment(U, count, ALG_PT2PT_RS);  // the wrapper's pt2pt_rs on the remainder
    } else if (sc.U > 0 && sc.U < count) {  // IN_PLACE: two pt2pt_rs calls
        if (!(rc = segment(0, sc.U, sc.forced))) rc = segment(sc.U, count, sc.forced);
    } else {
        rc = segment(0, count, sc.forced);
    }
    if (rc) return rc;
    return deliver ? dtype_unpack(res_all, count, t.dt, recvbuf) : 0;
}

// A two-level schedule across nodes (MPIR_Allreduce_two_level_MV2 / the two-level reduce helper):
// every node's partial from its ranks' operands (the node step's programs for local rank 0), then
// the leaders' programs over the partials.  Result: packed type-map bytes of elements [0, count)
// in res (device).
int run_two_level(const Operands &o, int count, const MnSched &sc, MPI_User_function *fn, char *res) {
    const Typed &t = o.t;
    const World &w = world();
    const int L = w.size, K = w.nnodes;
    HostBuf W(HS_OPERANDS), R(HS_RESULT), Pt(HS_PARTIALS);
    long rspan = 0;
    int rc = fetch(o, 0, count, W, rspan);
    if (rc) return rc;
    Pt.resize((size_t)rspan * (size_t)K + 1);
    R.resize((size_t)count * (size_t)t.tsize + 1);
    if (!Pt.data() || !R.data()) return MPI_ERR_NO_MEM;
    for (int j = 0; j < K; ++j) {
        char *nodeW = W.data() + (size_t)j * (size_t)L * (size_t)rspan, *part = Pt.data() + (size_t)j * rspan;
        if (L == 1) memcpy(part, nodeW, (size_t)rspan);
        else if ((rc = eval_into(sc.node.ps, 0, nodeW, rspan, 0, count, t, fn, part))) return rc;
    }
    if (K == 1) {
        rc = dtype_pack(Pt.data(), count, t.dt, R.data());
    } else if (sc.big) {  // more leaders than a program holds: the leaders' schedule itself
        BigEval ev{Pt.data(), rspan, K, count, &t, fn, true, {}};
        std::vector<char> out((size_t)rspan + 1);
        if (sc.forced == ALG_BINOMIAL) ev.binomial(sc.root, out.data());
        else if (sc.forced == ALG_KNOMIAL) ev.knomial(sc.root, sc.k, out.data());
        else if (sc.forced == ALG_REDSCAT_GATHER) ev.redscat_gather(out.data());
        else ev.rd(w.node, out.data());
        rc = dtype_pack(out.data(), count, t.dt, R.data());
    } else {
        rc = eval_range(sc.lead.ps, 0, Pt.data(), rspan, 0, count, t, fn, R.data());
    }
    if (rc) return rc;
    return mv2h_memcpy_htod(res, R.data(), (size_t)count * (size_t)t.tsize) ? MPI_ERR_OTHER : 0;
}

// every rank's plan_allreduce programs (forced as on this rank) equal `mine`
bool uniform_over_ranks(int n, int me, int count, const Typed &t, bool in_place, int forced, int opk,
                        const ProgSet &mine) {
    for (int j = 0; j < n; ++j) {
        if (j == me) continue;
        Plan q;
        if (plan_allreduce(n, j, (size_t)count, (int)t.tsize, (int)t.extent, in_place, forced, &q, opk)) return false;
        if (!same_progs(q.ps, mine)) return false;
    }
    return true;
}

// this rank's own programs over two ranges: [0, U) by a, [U, count) by b counted from U
int run_split2(const Operands &o, int count, const ProgSet &a, long U, const ProgSet &b, MPI_User_function *fn,
               void *recvbuf) {
    const Typed &t = o.t;
    char *res = dev_scratch(DS_RES_ALL, (size_t)count * (size_t)t.tsize);
    if (!res) return MPI_ERR_NO_MEM;
    HostBuf W(HS_OPERANDS), R(HS_RESULT);
    R.resize((size_t)count * (size_t)t.tsize + 1);
    if (!R.data()) return MPI_ERR_NO_MEM;
    long rspan = 0;
    int rc;
    if ((rc = fetch(o, 0, U, W, rspan)) || (rc = eval_range(a, 0, W.data(), rspan, 0, U, t, fn, R.data()))) return rc;
    if ((rc = fetch(o, U, count, W, rspan)) ||
        (rc = eval_range(b, U, W.data(), rspan, U, count, t, fn, R.data() + (size_t)U * t.tsize)))
        return rc;
    if (mv2h_memcpy_htod(res, R.data(), (size_t)count * (size_t)t.tsize)) return MPI_ERR_OTHER;
    return dtype_unpack(res, count, t.dt, recvbuf);
}

// MPIR_Allreduce_pt2pt_rd_MV2 (allreduce_osu.c:455-600) with its messages, on one node: each
// rank keeps its own accumulator in its host window and exchanges it with the step's partner
// through host shared memory, as the reference's ranks do through their shared-memory channel —
// the pre-step (an odd rank below 2 * rem reduces uop(tmp = x_{r-1}, acc)), log2(pof2) doubling
// steps (uop(tmp, acc) if commutative or the partner is lower, else uop(acc, tmp) copied back),
// the post-step (the even rank takes its partner's result).  The same operand order as the
// rank's own tree over every operand (the programs), with log2(pof2) uop calls instead of n - 1
// and one operand fetched instead of n.  Returns with *taken = false (and nothing done) when some
// rank's window or partner view could not be set up (a small /dev/shm): the caller takes the
// programs' path, on every rank alike.
int run_rd_exchange(const void *src, int count, const Typed &t, const HostOp &op, void *recvbuf, bool *taken) {
    World &w = world();
    const int n = w.size, me = w.rank;
    // MV2AMD_UOP_EXCHANGE: 1 always, 0 never; default from 4 ranks on, where it saves uop calls
    // (log2(pof2) against n - 1) and operand fetches (one against n); at 2 ranks both make one
    // call and the programs' path, whose operands never leave pinned memory, measured faster
    static const long mode = [] {
        const char *e = getenv("MV2AMD_UOP_EXCHANGE");
        return e && *e ? atol(e) : -1L;
    }();
    *taken = false;
    if (mode == 0 || (mode < 0 && n < 4)) return 0;
    const bool comm = op.opk != OPK_USER_NONCOMM;
    const size_t rspan = (size_t)dtype_span(t.dt, count), P = (size_t)count * (size_t)t.tsize;
    int pof2 = 1;
    while (pof2 * 2 <= n) pof2 *= 2;
    const int rem = n - pof2;
    const int newrank = me < 2 * rem ? ((me & 1) ? me / 2 : -1) : me - rem;
    auto real = [&](int q) { return q < rem ? 2 * q + 1 : q + rem; };
    // everything this rank needs is allocated before the vote, so that nothing after it can fail
    // short of a copy error (and that one still keeps the barriers: a rank leaving after the vote
    // would stall the others')
    const bool dev_src = mv2h_is_device_ptr(src), dev_dst = mv2h_is_device_ptr(recvbuf);
    // the operand's bytes from its true lower bound on (the layout is copied as it is, gaps
    // included: no pack / unpack on the host, whose block loop over a sparse span is slow)
    MPI_Aint tlb = 0, text = 0;
    PMPI_Type_get_true_extent(t.dt, &tlb, &text);
    const bool direct = tlb >= 0 && (t.contig || layout_on_device());
    const size_t dlen = direct ? rspan - (size_t)tlb : 0;
    HostBuf pk(HS_PACKED), T(HS_OPERANDS);
    pk.resize(P + 1);
    T.resize(rspan + 1);
    char *d = dev_src && !direct ? dev_scratch(DS_MINE, P) : nullptr;
    char *res = dev_scratch(DS_RES_ALL, P);
    char *sp = dev_dst && direct ? dev_scratch(DS_SPAN, rspan) : nullptr;
    char *acc = host_window(rspan + 1);
    bool ok = acc && pk.data() && T.data() && res && (d || !(dev_src && !direct)) && (sp || !(dev_dst && direct));
    host_barrier();  // every window reserved before any peer view is taken
    if (me < 2 * rem) ok = ok && host_peer_window((me & 1) ? me - 1 : me + 1, rspan + 1);
    if (newrank >= 0)
        for (int mask = 1; mask < pof2; mask <<= 1) ok = ok && host_peer_window(real(newrank ^ mask), rspan + 1);
    *taken = host_window_vote(ok);
    if (!*taken) return 0;
    auto peer = [&](int r) { return host_peer_window(r, rspan + 1); };
    auto uop = [&](const char *in, char *io) {
        int c = count;
        MPI_Datatype dd = t.dt;
        op.fn((void *)in, io, &c, &dd);
    };
    // this rank's operand into its window, in the type's layout.  From the vote on, a failing
    // copy or pack leaves rc set but the rank still takes part in every barrier below, so that
    // the other ranks finish the call (with this rank's stale window) instead of stalling
    PhaseClock pc;
    char *tmp = T.data();
    int rc = 0;
    if (direct) {
        if (dev_src) {
            if (dlen && mv2h_memcpy_dtoh(acc + tlb, (const char *)src + tlb, dlen)) rc = MPI_ERR_OTHER;
        } else {
            memcpy(acc + tlb, (const char *)src + tlb, dlen);
        }
    } else if (dev_src) {
        if (!(rc = dtype_pack(src, count, t.dt, d)) && P && mv2h_memcpy_dtoh(pk.data(), d, P)) rc = MPI_ERR_OTHER;
        if (!rc) rc = dtype_unpack(pk.data(), count, t.dt, acc);
    } else if (!(rc = dtype_pack(src, count, t.dt, pk.data()))) {
        rc = dtype_unpack(pk.data(), count, t.dt, acc);
    }
    pc.mark(UP_FETCH);
    // pre-step (:455-505)
    host_barrier();  // every accumulator in place
    if (me < 2 * rem && (me & 1)) memcpy(tmp, peer(me - 1), rspan);
    host_barrier();  // every read done before any accumulator changes
    if (me < 2 * rem && (me & 1)) uop(tmp, acc);
    // doubling steps (:507-584)
    for (int mask = 1; mask < pof2; mask <<= 1) {
        const int dst = newrank >= 0 ? real(newrank ^ mask) : -1;
        host_barrier();
        if (dst >= 0) memcpy(tmp, peer(dst), rspan);
        host_barrier();
        if (dst < 0) continue;
        if (comm || dst < me) {
            uop(tmp, acc);
        } else {
            uop(acc, tmp);
            memcpy(acc, tmp, rspan);
        }
    }
    // post-step (:585-600): the even rank below 2 * rem takes rank + 1's result
    host_barrier();
    if (me < 2 * rem && !(me & 1)) memcpy(tmp, peer(me + 1), rspan);
    const char *res_h = me < 2 * rem && !(me & 1) ? tmp : acc;
    if (!rc && direct && dev_dst) {  // the result's span up, its type map packed on the device
        if (dlen && mv2h_memcpy_htod(sp + tlb, res_h + tlb, dlen)) rc = MPI_ERR_OTHER;
        if (!rc) rc = dtype_pack(sp, count, t.dt, res);
    } else if (!rc && direct) {  // a host receive buffer: its type map from the result's
        dtype_merge_typemap((char *)recvbuf, res_h, t.dt, count);
    } else if (!rc) {
        rc = dtype_pack(res_h, count, t.dt, pk.data());
    }
    host_barrier();  // the post-step's reads are done before any window is reused
    pc.mark(UP_EVAL);  // the exchanges and the uop calls
    if (rc) return rc;
    if (!direct && P && mv2h_memcpy_htod(res, pk.data(), P)) return MPI_ERR_OTHER;
    // operand bytes this rank received (packed measure): pre- or post-step, and one per doubling step
    world().uop_in_bytes = P * (size_t)((me < 2 * rem) + (newrank >= 0 ? __builtin_ctz((unsigned)pof2) : 0));
    world().uop_area_bytes = rspan;
    rc = direct && !dev_dst ? 0 : dtype_unpack(res, count, t.dt, recvbuf);
    pc.mark(UP_DELIVER);
    return rc;
}

// one rank: recvbuf's type map <- src's
int copy_typemap(const void *src, void *recvbuf, int count, const Typed &t) {
    char *tmp = dev_scratch(DS_MINE, (size_t)count * (size_t)t.tsize);
    if (!tmp) return MPI_ERR_NO_MEM;
    const int rc = dtype_pack(src, count, t.dt, tmp);
    return rc ? rc : dtype_unpack(tmp, count, t.dt, recvbuf);
}

}  // namespace

int host_allreduce(const void *sendbuf, void *recvbuf, int count, MPI_Datatype dt, const HostOp &op) {
    const Job J = job();
    const Typed t = typed(dt);
    if (t.tsize < 0 || t.extent < 0) return MPI_ERR_TYPE;
    const int n = J.n, me = J.me;
    const bool in_place = sendbuf == MPI_IN_PLACE;
    const void *src = in_place ? recvbuf : sendbuf;
    if (n == 1) return in_place ? MPI_SUCCESS : copy_typemap(src, recvbuf, count, t);
    Plan p, rem;
    int rc, forced = 0;
    Split sp{&p.ps, 0, &p.ps, 0};
    if (J.multi) {
        MnSched sc;
        if ((rc = mn_host_schedule(MN_COLL_ALLREDUCE, (size_t)count, (int)t.tsize, (int)t.extent, in_place, op.opk, -1,
                                   &sc)))
            return rc == E_UNSUPPORTED ? MPI_ERR_UNSUPPORTED_OPERATION : MPI_ERR_INTERN;
        const bool whole = sc.kind == MN_TWO_LEVEL || sc.big || (sc.forced != ALG_RING && sc.U && sc.U < count);
        Operands o;
        if (whole && (rc = stage_operands(src, count, t, o))) return rc;
        if (sc.kind == MN_TWO_LEVEL) {
            char *res = dev_scratch(DS_RES_ALL, (size_t)count * (size_t)t.tsize);
            if (!res) return MPI_ERR_NO_MEM;
            if ((rc = run_two_level(o, count, sc, op.fn, res))) return rc;
            return dtype_unpack(res, count, t.dt, recvbuf);
        }
        if (sc.big) return run_big_flat(o, count, sc, op, recvbuf, true);
        p = sc.p;
        rem = sc.rem;
        forced = sc.forced;
        if (forced == ALG_RING) {  // ring chunks [0, U) are uniform, the remainder each rank's own
            sp = Split{&p.ps, sc.U, &rem.ps, sc.U};
        } else if (sc.U && sc.U < count) {  // IN_PLACE from 2 MiB: two pt2pt_rs calls, own programs
            return run_split2(o, count, p.ps, sc.U, rem.ps, op.fn, recvbuf);
        } else {
            sp = Split{&p.ps, uniform_over_ranks(n, me, count, t, in_place, forced, op.opk, p.ps) ? count : 0, &p.ps, 0};
        }
        return run_split(src, count, t, sp, op.fn, recvbuf, -1);
    }
    rc = plan_allreduce(n, me, (size_t)count, (int)t.tsize, (int)t.extent, in_place, 0, &p, op.opk);
    if (rc) return rc;
    pvar_note(PV_COLL_ALLREDUCE, p, in_place, (size_t)count, n);
    if (p.algo == ALG_RING) {
        // ring wrapper (allreduce_osu.c:3758-3818): the ring over (count / n) * n elements unless
        // IN_PLACE, pt2pt_rs (recursive doubling for user ops) on the rest
        sp.U = in_place ? 0 : (long)(count / n) * n;
        if (sp.U < count) {
            rc = plan_allreduce(n, me, (size_t)(count - sp.U), (int)t.tsize, (int)t.extent, in_place, ALG_PT2PT_RS, &rem,
                                op.opk);
            if (rc) return rc;
            sp.own = &rem.ps;
            sp.own_base = sp.U;
            if (sp.U == 0 && rem.algo == ALG_PT2PT_RD) {  // the wrapper's pt2pt_rs is recursive doubling
                bool taken = false;
                rc = run_rd_exchange(src, count, t, op, recvbuf, &taken);
                if (taken) return rc;
            }
        }
    } else {
        sp.U = uniform_over_ranks(n, me, count, t, in_place, 0, op.opk, p.ps) ? count : 0;
        if (sp.U == 0 && p.algo == ALG_PT2PT_RD && count > 0) {  // every rank its own tree: the exchanges
            bool taken = false;
            rc = run_rd_exchange(src, count, t, op, recvbuf, &taken);
            if (taken) return rc;
        }
    }
    return run_split(src, count, t, sp, op.fn, recvbuf, -1);
}

// MPI_Reduce: the root's programs (MPIR_Reduce_index_tuned_intra_MV2's choice, binomial /
// knomial / shmem / ...) evaluated over ranges split across every rank
int host_reduce(const void *sendbuf, void *recvbuf, int count, MPI_Datatype dt, const HostOp &op, int root) {
    const Job J = job();
    const Typed t = typed(dt);
    if (t.tsize < 0 || t.extent < 0) return MPI_ERR_TYPE;
    const int n = J.n, me = J.me;
    const void *src = sendbuf == MPI_IN_PLACE ? recvbuf : sendbuf;
    if (n == 1) return sendbuf == MPI_IN_PLACE ? MPI_SUCCESS : copy_typemap(src, recvbuf, count, t);
    Plan p, pr;
    int rc;
    if (J.multi) {
        MnSched sc;
        if ((rc = mn_host_schedule(MN_COLL_REDUCE, (size_t)count, (int)t.tsize, (int)t.extent, sendbuf == MPI_IN_PLACE,
                                   op.opk, root, &sc)))
            return rc == E_UNSUPPORTED ? MPI_ERR_UNSUPPORTED_OPERATION : MPI_ERR_INTERN;
        if (sc.kind == MN_TWO_LEVEL || sc.big) {
            Operands o;
            if ((rc = stage_operands(src, count, t, o))) return rc;
            if (sc.big) return run_big_flat(o, count, sc, op, recvbuf, me == root);
            if (me != root) return MPI_SUCCESS;  // only the root's result counts: the root evaluates it
            char *res = dev_scratch(DS_RES_ALL, (size_t)count * (size_t)t.tsize);
            if (!res) return MPI_ERR_NO_MEM;
            if ((rc = run_two_level(o, count, sc, op.fn, res))) return rc;
            return dtype_unpack(res, count, t.dt, recvbuf);
        }
        pr = sc.p;  // the root's programs of the flat algorithm over the job's ranks
        const Split sp{&pr.ps, count, &pr.ps, 0};
        return run_split(src, count, t, sp, op.fn, recvbuf, root);
    }
    rc = plan_reduce(n, me, root, (size_t)count, (int)t.tsize, (int)t.extent, &p, op.opk);
    if (rc) return rc;
    pvar_note(PV_COLL_REDUCE, p, sendbuf == MPI_IN_PLACE, (size_t)count, n);  // every rank runs the algorithm
    if ((rc = plan_reduce(n, root, root, (size_t)count, (int)t.tsize, (int)t.extent, &pr, op.opk))) return rc;
    const Split sp{&pr.ps, count, &pr.ps, 0};
    return run_split(src, count, t, sp, op.fn, recvbuf, root);
}

// Reduce_scatter: the order of MPIR_Reduce_scatter_MV2's choice for this rank's block — ring,
// recursive halving, pairwise or reduce + scatter for commutative ops,
// MPIR_Reduce_scatter_non_comm_MV2 (mirror-permuted halving or recursive doubling) for
// non-commutative ones, which MPI_Ireduce_scatter and both block forms choose alike
// (orders.cpp plan_rs_noncomm).  Each rank evaluates its own block (above kMaxRanks ranks from
// the algorithm's message schedule or expression tree, BigEval).
int host_reduce_scatter(const void *sendbuf, void *recvbuf, const int *counts, MPI_Datatype dt, const HostOp &op) {
    const Job J = job();
    const Typed t = typed(dt);
    if (t.tsize < 0 || t.extent <= 0) return MPI_ERR_TYPE;
    const int n = J.n, me = J.me;
    // across nodes MV2AMD_MN_PROG_MAX may lower the programs' limit (runtime/coll.cpp mn_prog_max)
    const int pm = world().nnodes > 1 ? mn_prog_max() : kMaxRanks;
    long total = 0, disp = 0;
    std::vector<size_t> cz(n);
    for (int j = 0; j < n; ++j) {
        if (j == me) disp = total;
        total += counts[j];
        cz[j] = (size_t)counts[j];
    }
    ProgSet ps{};
    Plan p;
    int rc;
    const bool noncomm = op.opk == OPK_USER_NONCOMM;
    if (n > pm && noncomm) {
        // MPIR_Reduce_scatter_non_comm_MV2 (red_scat_osu.c:1367-1760) and the nonblocking / block
        // forms' same choice (orders.cpp plan_rs_noncomm) beyond a program's registers: this rank's
        // block evaluated from the algorithm's expression; a power-of-two size with equal counts
        // takes the mirror-permuted halving, else recursive doubling
        bool equal = true;
        for (int j = 1; j < n; ++j) equal = equal && counts[j] == counts[0];
        p.algo = (n & (n - 1)) == 0 && equal ? ALG_RS_NONCOMM_POF2 : ALG_RS_NONCOMM_RD;
        if (nbc_kind() == NBC_NONE) pvar_note(PV_COLL_REDUCE_SCATTER, p, false, (size_t)total, n);
    } else if (n > pm) {
        // more ranks than a program holds: the algorithm's schedule evaluated for this rank's block
        const int algo = reduce_scatter_algo(n, total * t.tsize);
        p.algo = algo;
        const int id = algo == ALG_RS_RING ? PV_RS_RING : algo == ALG_RS_PAIRWISE ? PV_RS_PAIRWISE : PV_RS_REC_HALVING;
        const int chain[3] = {PV_RS_BASIC, PV_RED_TWO_LEVEL_HELPER, PV_RED_BINOMIAL};
        if (algo == ALG_RS_BASIC) pvar_note_ids(chain, world().rank == 0 ? 3 : 2);
        else pvar_note_ids(&id, 1);
    } else {
        if ((rc = plan_reduce_scatter(n, me, cz.data(), (int)t.tsize, (int)t.extent, &p, op.opk))) return rc;
        if (J.multi && p.algo == ALG_RS_BASIC) {  // the reduce inside is the multi-node one
            const int chain[3] = {PV_RS_BASIC, PV_RED_TWO_LEVEL_HELPER, PV_RED_BINOMIAL};
            pvar_note_ids(chain, world().rank == 0 ? 3 : 2);
        } else {
            pvar_note(PV_COLL_REDUCE_SCATTER, p, false, (size_t)total, n);
        }
        ps = p.ps;
    }
    // each rank receives only its own block of every operand (an all-to-all of blocks), except the
    // multi-node basic algorithm, whose reduce every rank evaluates whole
    const bool basic_mn = J.multi && op.opk != OPK_USER_NONCOMM && p.algo == ALG_RS_BASIC;
    Operands o;
    {
        const void *src = sendbuf == MPI_IN_PLACE ? recvbuf : sendbuf;
        if (basic_mn) {
            rc = stage_operands(src, (int)total, t, o);
        } else {
            char *mine = nullptr;
            std::vector<long> lo((size_t)n), hi((size_t)n);
            for (long j = 0, d = 0; j < n; d += counts[j], ++j) {
                lo[j] = d;
                hi[j] = d + counts[j];
            }
            if (!(rc = pack_mine(src, (int)total, t, &mine))) rc = exchange_ranges(mine, (int)total, t, lo, hi, o);
        }
        if (rc) return rc;
    }
    const int c = counts[me];
    if (basic_mn) {
        // MPIR_Reduce_Scatter_Basic_MV2 (red_scat_osu.c:300-413): MPIR_Reduce_MV2 to rank 0 over the
        // whole job — the two-level reduce helper for a commutative op — then the scatter: every
        // rank evaluates that reduce's result (a basic operand is at most a few hundred bytes)
        MnSched sc;
        if ((rc = mn_host_schedule(MN_COLL_REDUCE, (size_t)total, (int)t.tsize, (int)t.extent, false, op.opk, 0, &sc)))
            return rc == E_UNSUPPORTED ? MPI_ERR_UNSUPPORTED_OPERATION : MPI_ERR_INTERN;
        if (c == 0) return MPI_SUCCESS;
        char *res = dev_scratch(DS_RES_ALL, (size_t)total * (size_t)t.tsize);
        if (!res) return MPI_ERR_NO_MEM;
        if (sc.kind != MN_TWO_LEVEL || (rc = run_two_level(o, (int)total, sc, op.fn, res))) return rc ? rc : MPI_ERR_INTERN;
        return dtype_unpack(res + (size_t)disp * (size_t)t.tsize, c, t.dt, recvbuf);
    }
    if (c == 0) return MPI_SUCCESS;
    HostBuf W(HS_OPERANDS), R(HS_RESULT);
    long rspan = 0;
    if ((rc = fetch(o, disp, disp + c, W, rspan))) return rc;
    R.resize((size_t)c * (size_t)t.tsize + 1);
    if (!R.data()) return MPI_ERR_NO_MEM;
    if (n > pm && noncomm) {
        // the expression's tree over the n operands' block, uop(in = b, inout = a) per node
        std::vector<ExprNode> nodes;
        const int root = rs_noncomm_expr(n, me, p.algo == ALG_RS_NONCOMM_POF2, nodes);
        BigEval ev{W.data(), rspan, n, c, &t, op.fn, false, {}};
        std::vector<char> out((size_t)rspan + 1);
        ev.expr(nodes, root, 0, out.data());
        if ((rc = dtype_pack(out.data(), c, t.dt, R.data()))) return rc;
        return dtype_unpack(R.data(), c, t.dt, recvbuf);
    }
    if (n > pm) {
        BigEval ev{W.data(), rspan, n, c, &t, op.fn, true, {}};
        std::vector<char> out((size_t)rspan + 1);
        if (p.algo == ALG_RS_RING) ev.rs_ring(me, out.data());
        else if (p.algo == ALG_RS_PAIRWISE) ev.rs_pairwise(me, out.data());
        else ev.rs_halving(me, out.data());
        if ((rc = dtype_pack(out.data(), c, t.dt, R.data()))) return rc;
        return dtype_unpack(R.data(), c, t.dt, recvbuf);
    }
    if ((rc = eval_range(ps, 0, W.data(), rspan, disp, disp + c, t, op.fn, R.data()))) return rc;
    return dtype_unpack(R.data(), c, t.dt, recvbuf);
}

}  // namespace mv2

namespace {
// the hook's user function: inout = 2 in + 3 inout, int32 wrapping (neither commutative nor
// associative, so every operand order shows)
void hook_fn(void *in, void *inout, int *len, MPI_Datatype *) {
    const int32_t *a = (const int32_t *)in;
    int32_t *b = (int32_t *)inout;
    for (int i = 0; i < *len; ++i) b[i] = (int32_t)((uint32_t)a[i] * 2u + (uint32_t)b[i] * 3u);
}
}  // namespace

extern "C" int mv2h_host_sched_eval(int form, int n, int me, int root, int k, int count, int commute,
                                    const int32_t *ops, int32_t *out) {
    using namespace mv2;
    if (n < 1 || count < 1 || me < 0 || me >= n || root < 0 || root >= n || !ops || !out) return MPI_ERR_ARG;
    const Typed t = typed(MPI_INT);
    BigEval ev{(const char *)ops, (long)count * 4, n, count, &t, hook_fn, commute != 0, {}};
    char *o = (char *)out;
    switch (form) {
        case MV2H_SCHED_RD: ev.rd(me, o); break;
        case MV2H_SCHED_PT2PT_RS: ev.rs(o); break;
        case MV2H_SCHED_BINOMIAL: ev.binomial(root, o); break;
        case MV2H_SCHED_KNOMIAL: ev.knomial(root, k, o); break;
        case MV2H_SCHED_REDSCAT_GATHER: ev.redscat_gather(o); break;
        case MV2H_SCHED_RS_HALVING: ev.rs_halving(me, o); break;
        case MV2H_SCHED_RS_PAIRWISE: ev.rs_pairwise(me, o); break;
        case MV2H_SCHED_RS_RING: ev.rs_ring(me, o); break;
        case MV2H_SCHED_RING_CHUNK: ev.ring_chunk(me, o); break;
        case MV2H_SCHED_RS_NONCOMM: {  // equal blocks: the mirror-permuted halving at a power of two
            std::vector<ExprNode> nodes;
            const int e = rs_noncomm_expr(n, me, (n & (n - 1)) == 0, nodes);
            if (e < 0) return MPI_ERR_INTERN;
            ev.expr(nodes, e, 0, o);
            break;
        }
        default: return MPI_ERR_ARG;
    }
    return 0;
}
