// datatype.cpp — derived datatypes (contiguous, vector, hvector,
// indexed_block, nested) and MPI_Pack / MPI_Unpack.
//
// A committed type is flattened into the (offset, length) byte segments of
// one element (the reference builds a dataloop tree and walks it with the
// segment stack machine: dataloop_create_vector.c:27, segment.c:344,
// segment_packunpack.c:175-305).  Device buffers are packed by HIP kernels:
// a regular layout (equal lengths at a constant stride, the MPI_Type_vector
// case) is one strided pack/unpack launch (mv2h_pack_strided), replacing
// MPID_Segment_pack_device (ibv_cuda_util.c:623) and its cudaMemcpy2DAsync /
// pack_unpack_vector_kernel paths (pack_unpack.cu:419); every other layout
// (pair types, indexed blocks, vectors with count > 1, nested types) is one
// run-table launch (mv2h_pack_segments).  Host buffers are copied on the
// host, as the reference does for host memory.
#include "datatype.h"

#include <string.h>

#include <mutex>
#include <vector>

#include "../../../include/mv2h.h"
#include "../common.h"
#include "../runtime/world.h"

namespace {

struct Seg {
    long off, len;
};

struct Derived {
    bool live = false, committed = false;
    long size = 0, lb = 0, extent = 0, true_lb = 0, true_extent = 0;
    long align = 1;         // alignsize (mpid_type_struct.c:42-124)
    std::vector<Seg> segs;  // one element, sorted by construction order, merged
    // layout summary, computed once (pack calls then cost O(1) host work): one element is
    // reg_n blocks of reg_blk bytes at reg_stride from offset 0
    bool summarised = false, reg = false;
    long reg_n = 0, reg_blk = 0, reg_stride = 0;
};

std::vector<Derived> g_types;
std::recursive_mutex g_mu;
constexpr int kDerivedBase = (int)0x8c000010;

Derived *derived(MPI_Datatype dt) {
    const unsigned idx = (unsigned)(dt - kDerivedBase);
    if (((unsigned)dt & 0xfc000000u) != 0x8c000000u || idx >= g_types.size() || !g_types[idx].live) return nullptr;
    return &g_types[idx];
}

// segments of one element of any (builtin or derived) type
bool type_segs(MPI_Datatype dt, std::vector<Seg> &out, long &extent, long &size) {
    if (const mv2::DtypeInfo *b = mv2::dtype_lookup(dt)) {
        out.assign(1, Seg{0, b->size});
        if (b->size != b->extent) {
            // pair types: value and loc fields (padding is not data)
            out.clear();
            if (dt == (int)0x8c000003) out = {Seg{0, 2}, Seg{4, 4}};           // SHORT_INT
            else if (dt == (int)0x8c000004) out = {Seg{0, 10}, Seg{16, 4}};    // LONG_DOUBLE_INT
            else out = {Seg{0, 12}};                                           // DOUBLE_INT, LONG_INT
        }
        extent = b->extent;
        size = b->size;
        return true;
    }
    Derived *d = derived(dt);
    if (!d) return false;
    out = d->segs;
    extent = d->extent;
    size = d->size;
    return true;
}

void push_merge(std::vector<Seg> &v, Seg s) {
    if (s.len <= 0) return;
    if (!v.empty() && v.back().off + v.back().len == s.off) v.back().len += s.len;
    else v.push_back(s);
}

// One block of a type map: `blocklen` copies of `old` starting at byte `disp`.
struct Block {
    long disp;
    long blocklen;
    MPI_Datatype old;
};

// lb / ub of a (builtin or derived) type, as MPI_Type_get_extent reports them
bool type_bounds(MPI_Datatype dt, long &lb, long &extent);

// alignsize of a type (MPID_Type_struct_alignsize, mpid_type_struct.c:42-124,
// with the x86-64 configure results: fp types aligned to their size up to 16,
// everything else up to 8; pair types = the larger member, pairtype.c:26)
long type_align(MPI_Datatype dt) {
    if (const mv2::DtypeInfo *b = mv2::dtype_lookup(dt)) {
        switch ((unsigned)dt) {
        case 0x4c00040au: case 0x4c00080bu: case 0x4c00100cu: return b->size;  // FLOAT DOUBLE LONG_DOUBLE
        case 0x8c000000u: return 4;   // FLOAT_INT
        case 0x8c000001u: return 8;   // DOUBLE_INT
        case 0x8c000002u: return 8;   // LONG_INT
        case 0x8c000003u: return 4;   // SHORT_INT
        case 0x8c000004u: return 16;  // LONG_DOUBLE_INT
        default: return b->size < 8 ? b->size : 8;
        }
    }
    Derived *d = derived(dt);
    return d ? d->align : 1;
}

// General constructor (every MPI_Type_* constructor reduces to this, like the
// reference's dataloop constructors reduce to DLOOP_Dataloop_create_struct,
// dataloop_create_struct.c): the element's segments are the blocks' segments in
// type-map order, merged when adjacent; lb/ub follow MPI-3.1 §4.1.6 (blocks
// of length 0 do not count, zero-blklen-vector.c); size = sum of block sizes.
int make_struct(const std::vector<Block> &blocks, MPI_Datatype *out, bool pad = false) {
    std::lock_guard<std::recursive_mutex> lk(g_mu);
    Derived d;
    d.live = true;
    d.align = 1;
    long lo = 0, hi = 0, lb = 0, ub = 0;
    bool any_seg = false, any_blk = false;
    for (const Block &b : blocks) {
        if (b.blocklen < 0) return MPI_ERR_ARG;
        std::vector<Seg> os;
        long oext = 0, osize = 0, olb = 0, oext2 = 0;
        if (!type_segs(b.old, os, oext, osize) || !type_bounds(b.old, olb, oext2)) return MPI_ERR_TYPE;
        if (type_align(b.old) > d.align) d.align = type_align(b.old);
        if (b.blocklen == 0) continue;
        for (long k = 0; k < b.blocklen; ++k)
            for (const Seg &sg : os) {
                const Seg t{b.disp + k * oext + sg.off, sg.len};
                if (t.len <= 0) continue;
                push_merge(d.segs, t);
                if (!any_seg || t.off < lo) lo = t.off;
                if (!any_seg || t.off + t.len > hi) hi = t.off + t.len;
                any_seg = true;
            }
        const long b0 = b.disp + olb, b1 = b.disp + olb + b.blocklen * oext;
        if (!any_blk || b0 < lb) lb = b0;
        if (!any_blk || b1 > ub) ub = b1;
        any_blk = true;
        d.size += b.blocklen * osize;
    }
    d.true_lb = any_seg ? lo : 0;
    d.true_extent = any_seg ? hi - lo : 0;
    if (d.true_lb < 0) return MPI_ERR_ARG;  // data below the buffer pointer: not supported
    d.lb = any_blk ? lb : 0;
    d.extent = any_blk ? ub - lb : 0;
    if (pad && d.align > 1 && d.extent % d.align)  // struct padding (mpid_type_struct.c:400-411)
        d.extent += d.align - d.extent % d.align;
    g_types.push_back(d);
    *out = kDerivedBase + (int)(g_types.size() - 1);
    return MPI_SUCCESS;
}

int make_type(const std::vector<long> &block_offsets, int blocklen, MPI_Datatype old, MPI_Datatype *out) {
    std::vector<Block> blocks;
    blocks.reserve(block_offsets.size());
    for (long bo : block_offsets) blocks.push_back(Block{bo, blocklen, old});
    return make_struct(blocks, out);
}

void summarise(Derived *d) {
    if (d->summarised) return;
    d->summarised = true;
    const auto &s = d->segs;
    d->reg = false;
    if (s.empty() || s[0].off != 0) return;
    const long blk = s[0].len, stride = s.size() > 1 ? s[1].off - s[0].off : d->extent;
    for (size_t i = 0; i < s.size(); ++i)
        if (s[i].len != blk || s[i].off != (long)i * stride) return;
    d->reg = stride >= blk;
    d->reg_n = (long)s.size();
    d->reg_blk = blk;
    d->reg_stride = stride;
}

// regular layout of `count` elements: nblocks x blk bytes at constant stride
bool regular(Derived *d, long extent, int count, long &nblocks, long &blk, long &stride) {
    summarise(d);
    if (!d->reg) return false;
    blk = d->reg_blk;
    stride = d->reg_n > 1 ? d->reg_stride : extent;
    if (count > 1 && d->reg_n * stride != extent) return false;
    nblocks = d->reg_n * count;
    return stride >= blk;
}

int pack_impl(const char *in, int count, MPI_Datatype dt, char *out, bool unpack) {
    // a derived type's segments are used in place (no per-call copy of a large type map)
    std::vector<Seg> bsegs;
    long ext = 0, size = 0;
    Derived *d = derived(dt);
    if (d) {
        ext = d->extent;
        size = d->size;
    } else if (!type_segs(dt, bsegs, ext, size)) {
        return MPI_ERR_TYPE;
    }
    const std::vector<Seg> &segs = d ? d->segs : bsegs;
    const bool din = mv2h_is_device_ptr(in), dout = mv2h_is_device_ptr(out);
    if (!din && !dout) {
        // host <-> host: reference semantics, host copies; a regular layout (vectors) moves
        // fixed-size blocks without a call per block
        long nb = 0, blk = 0, stride = 0;
        if (d && regular(d, ext, count, nb, blk, stride) && (blk == 4 || blk == 8 || blk == 16 || blk == 32)) {
            for (long i = 0; i < nb; ++i) {
                char *dst = unpack ? out + i * stride : out + i * blk;
                const char *src = unpack ? in + i * blk : in + i * stride;
                switch (blk) {
                case 4: memcpy(dst, src, 4); break;
                case 8: memcpy(dst, src, 8); break;
                case 16: memcpy(dst, src, 16); break;
                default: memcpy(dst, src, 32); break;
                }
            }
            return MPI_SUCCESS;
        }
        if (segs.size() == 1 && segs[0].off == 0 && segs[0].len == ext) {  // contiguous
            memcpy(out, in, (size_t)count * ext);
            return MPI_SUCCESS;
        }
        long pos = 0;
        for (int e = 0; e < count; ++e)
            for (const Seg &s : segs) {
                if (!unpack) memcpy(out + pos, in + (long)e * ext + s.off, s.len);
                else memcpy(out + (long)e * ext + s.off, in + pos, s.len);
                pos += s.len;
            }
        return MPI_SUCCESS;
    }
    if (!din || !dout) {
        // mixed: stage the host side on the device so that the layout work runs on the GPU
        const long span = count ? (long)(count - 1) * ext + (d ? d->true_lb + d->true_extent : ext) : 0;
        const long packed = (long)count * size;
        // device staging from the pool (runtime/world.cpp pool_get): no hipMalloc / hipFree per call
        void *tmp = nullptr;
        int rc;
        if (!unpack) {
            // pack: src strided, dst packed
            if (!din) {
                if (!(tmp = mv2::pool_get(span))) return MPI_ERR_NO_MEM;
                mv2h_memcpy_htod(tmp, in, span);
                rc = pack_impl((const char *)tmp, count, dt, out, false);
            } else {
                if (!(tmp = mv2::pool_get(packed))) return MPI_ERR_NO_MEM;
                rc = pack_impl(in, count, dt, (char *)tmp, false);
                if (!rc) mv2h_memcpy_dtoh(out, tmp, packed);
            }
        } else if (!din) {
            if (!(tmp = mv2::pool_get(packed))) return MPI_ERR_NO_MEM;
            mv2h_memcpy_htod(tmp, in, packed);
            rc = pack_impl((const char *)tmp, count, dt, out, true);
        } else {
            // unpack into a host destination: copy its current bytes so gaps survive
            if (!(tmp = mv2::pool_get(span))) return MPI_ERR_NO_MEM;
            mv2h_memcpy_htod(tmp, out, span);
            rc = pack_impl(in, count, dt, (char *)tmp, true);
            if (!rc) mv2h_memcpy_dtoh(out, tmp, span);
        }
        mv2::pool_put(tmp);
        return rc;
    }
    // device <-> device
    long nb = 0, blk = 0, stride = 0;
    if (d && regular(d, ext, count, nb, blk, stride)) {
        int rc = unpack ? mv2h_unpack_strided(in, out, nb, blk, stride, nullptr)
                        : mv2h_pack_strided(in, out, nb, blk, stride, nullptr);
        return rc ? MPI_ERR_OTHER : MPI_SUCCESS;
    }
    if (segs.size() == 1 && segs[0].off == 0 && segs[0].len == ext)  // contiguous
        return mv2h_memcpy_dtod(out, in, (size_t)count * ext) ? MPI_ERR_OTHER : MPI_SUCCESS;
    // every other layout (pair types, indexed, vectors with count > 1, nested): one launch
    std::vector<int64_t> offs(segs.size()), lens(segs.size());
    for (size_t i = 0; i < segs.size(); ++i) {
        offs[i] = segs[i].off;
        lens[i] = segs[i].len;
    }
    return mv2h_pack_segments(in, out, (size_t)count, (size_t)ext, offs.data(), lens.data(), (int)segs.size(),
                              unpack ? 1 : 0, nullptr)
               ? MPI_ERR_OTHER
               : MPI_SUCCESS;
}

}  // namespace

bool dtype_valid(MPI_Datatype dt) { return mv2::dtype_lookup(dt) != nullptr || derived(dt) != nullptr; }
bool dtype_is_builtin(MPI_Datatype dt) { return mv2::dtype_lookup(dt) != nullptr; }
bool dtype_committed(MPI_Datatype dt) {
    if (mv2::dtype_lookup(dt)) return true;
    Derived *d = derived(dt);
    return d && d->committed;
}
long dtype_true_lb(MPI_Datatype dt) {
    Derived *d = derived(dt);
    return d ? d->true_lb : 0;
}
bool dtype_is_contiguous(MPI_Datatype dt) {
    // builtin pair types carry padding; copying it with the data is harmless for movement-only collectives
    if (mv2::dtype_lookup(dt)) return true;
    Derived *d = derived(dt);
    return d && d->segs.size() <= 1 && d->size == d->extent;
}
long dtype_size(MPI_Datatype dt) {
    if (const mv2::DtypeInfo *b = mv2::dtype_lookup(dt)) return b->size;
    Derived *d = derived(dt);
    return d ? d->size : -1;
}
long dtype_extent(MPI_Datatype dt) {
    if (const mv2::DtypeInfo *b = mv2::dtype_lookup(dt)) return b->extent;
    Derived *d = derived(dt);
    return d ? d->extent : -1;
}
template <size_t B>
static void copy_blocks(char *dst, const char *src, long nblocks, long stride) {
    for (long i = 0; i < nblocks; ++i) memcpy(dst + i * stride, src + i * stride, B);
}

void dtype_merge_typemap(char *dst, const char *src, MPI_Datatype dt, long count) {
    std::lock_guard<std::recursive_mutex> lk(g_mu);
    if (Derived *d = derived(dt)) {
        // regular layouts (vectors): fixed-size block copies, no per-block call
        long nb = 0, blk = 0, stride = 0;
        if (count > 0 && regular(d, d->extent, (int)count, nb, blk, stride)) {
            switch (blk) {
            case 4: copy_blocks<4>(dst, src, nb, stride); return;
            case 8: copy_blocks<8>(dst, src, nb, stride); return;
            case 16: copy_blocks<16>(dst, src, nb, stride); return;
            case 32: copy_blocks<32>(dst, src, nb, stride); return;
            default: break;
            }
        }
    }
    std::vector<Seg> segs;
    long extent = 0, size = 0;
    if (!type_segs(dt, segs, extent, size)) return;
    for (long e = 0; e < count; ++e)
        for (const Seg &sg : segs) memcpy(dst + e * extent + sg.off, src + e * extent + sg.off, (size_t)sg.len);
}

int dtype_pack(const void *in, int count, MPI_Datatype dt, void *out) {
    std::lock_guard<std::recursive_mutex> lk(g_mu);
    return count > 0 ? pack_impl((const char *)in, count, dt, (char *)out, false) : MPI_SUCCESS;
}
int dtype_unpack(const void *in, int count, MPI_Datatype dt, void *out) {
    std::lock_guard<std::recursive_mutex> lk(g_mu);
    return count > 0 ? pack_impl((const char *)in, count, dt, (char *)out, true) : MPI_SUCCESS;
}

long dtype_span(MPI_Datatype dt, int count) {
    if (count <= 0) return 0;
    if (const mv2::DtypeInfo *b = mv2::dtype_lookup(dt)) return (long)count * b->extent;
    Derived *d = derived(dt);
    if (!d) return -1;
    return (long)(count - 1) * d->extent + d->true_lb + d->true_extent;
}

namespace {
bool type_bounds(MPI_Datatype dt, long &lb, long &extent) {
    if (const mv2::DtypeInfo *b = mv2::dtype_lookup(dt)) {
        lb = 0;
        extent = b->extent;
        return true;
    }
    Derived *d = derived(dt);
    if (!d) return false;
    lb = d->lb;
    extent = d->extent;
    return true;
}
}  // namespace

#define WEAK(name) __attribute__((weak, alias("P" #name)))

extern "C" {

int PMPI_Type_size(MPI_Datatype dt, int *size) {
    long s = dtype_size(dt);
    if (s < 0) return MPI_ERR_TYPE;
    *size = (int)s;
    return MPI_SUCCESS;
}
int MPI_Type_size(MPI_Datatype dt, int *size) WEAK(MPI_Type_size);

int PMPI_Type_get_extent(MPI_Datatype dt, MPI_Aint *lb, MPI_Aint *extent) {
    long e = dtype_extent(dt);
    if (e < 0) return MPI_ERR_TYPE;
    Derived *d = derived(dt);
    *lb = d ? d->lb : 0;
    *extent = e;
    return MPI_SUCCESS;
}
int MPI_Type_get_extent(MPI_Datatype dt, MPI_Aint *lb, MPI_Aint *extent) WEAK(MPI_Type_get_extent);

int PMPI_Type_get_true_extent(MPI_Datatype dt, MPI_Aint *tlb, MPI_Aint *text) {
    if (const mv2::DtypeInfo *b = mv2::dtype_lookup(dt)) {
        *tlb = 0;
        *text = b->size == b->extent ? b->extent : (dt == (int)0x8c000003 ? 8 : b->extent - 4);
        return MPI_SUCCESS;
    }
    Derived *d = derived(dt);
    if (!d) return MPI_ERR_TYPE;
    *tlb = d->true_lb;
    *text = d->true_extent;
    return MPI_SUCCESS;
}
int MPI_Type_get_true_extent(MPI_Datatype dt, MPI_Aint *tlb, MPI_Aint *text) WEAK(MPI_Type_get_true_extent);

int PMPI_Type_contiguous(int count, MPI_Datatype old, MPI_Datatype *nt) {
    if (count < 0) return MPI_ERR_COUNT;
    std::vector<Seg> s;
    long ext = 0, sz = 0;
    if (!type_segs(old, s, ext, sz)) return MPI_ERR_TYPE;
    std::vector<long> offs;
    for (int i = 0; i < count; ++i) offs.push_back((long)i * ext);
    return make_type(offs, 1, old, nt);
}
int MPI_Type_contiguous(int count, MPI_Datatype old, MPI_Datatype *nt) WEAK(MPI_Type_contiguous);

int PMPI_Type_create_hvector(int count, int blocklen, MPI_Aint stride, MPI_Datatype old, MPI_Datatype *nt) {
    if (count < 0) return MPI_ERR_COUNT;
    std::vector<long> offs;
    for (int i = 0; i < count; ++i) offs.push_back((long)i * stride);
    return make_type(offs, blocklen, old, nt);
}
int MPI_Type_create_hvector(int count, int blocklen, MPI_Aint stride, MPI_Datatype old, MPI_Datatype *nt) WEAK(MPI_Type_create_hvector);

int PMPI_Type_vector(int count, int blocklen, int stride, MPI_Datatype old, MPI_Datatype *nt) {
    std::vector<Seg> s;
    long ext = 0, sz = 0;
    if (!type_segs(old, s, ext, sz)) return MPI_ERR_TYPE;
    return PMPI_Type_create_hvector(count, blocklen, (MPI_Aint)stride * ext, old, nt);
}
int MPI_Type_vector(int count, int blocklen, int stride, MPI_Datatype old, MPI_Datatype *nt) WEAK(MPI_Type_vector);

int PMPI_Type_create_indexed_block(int count, int blocklen, const int displs[], MPI_Datatype old, MPI_Datatype *nt) {
    if (count < 0) return MPI_ERR_COUNT;
    std::vector<Seg> s;
    long ext = 0, sz = 0;
    if (!type_segs(old, s, ext, sz)) return MPI_ERR_TYPE;
    std::vector<long> offs;
    for (int i = 0; i < count; ++i) offs.push_back((long)displs[i] * ext);
    return make_type(offs, blocklen, old, nt);
}
int MPI_Type_create_indexed_block(int count, int blocklen, const int displs[], MPI_Datatype old, MPI_Datatype *nt) WEAK(MPI_Type_create_indexed_block);

int PMPI_Type_create_hindexed_block(int count, int blocklen, const MPI_Aint displs[], MPI_Datatype old,
                                    MPI_Datatype *nt) {
    if (count < 0) return MPI_ERR_COUNT;
    std::vector<long> offs(displs, displs + count);
    return make_type(offs, blocklen, old, nt);
}
int MPI_Type_create_hindexed_block(int count, int blocklen, const MPI_Aint displs[], MPI_Datatype old,
                                   MPI_Datatype *nt) WEAK(MPI_Type_create_hindexed_block);

int PMPI_Type_indexed(int count, const int blocklens[], const int displs[], MPI_Datatype old, MPI_Datatype *nt) {
    if (count < 0) return MPI_ERR_COUNT;
    long lb = 0, ext = 0;
    if (!type_bounds(old, lb, ext)) return MPI_ERR_TYPE;
    std::vector<Block> blocks;
    for (int i = 0; i < count; ++i) blocks.push_back(Block{(long)displs[i] * ext, blocklens[i], old});
    return make_struct(blocks, nt);
}
int MPI_Type_indexed(int count, const int blocklens[], const int displs[], MPI_Datatype old, MPI_Datatype *nt) WEAK(MPI_Type_indexed);

int PMPI_Type_create_hindexed(int count, const int blocklens[], const MPI_Aint displs[], MPI_Datatype old,
                              MPI_Datatype *nt) {
    if (count < 0) return MPI_ERR_COUNT;
    if (!dtype_valid(old)) return MPI_ERR_TYPE;
    std::vector<Block> blocks;
    for (int i = 0; i < count; ++i) blocks.push_back(Block{(long)displs[i], blocklens[i], old});
    return make_struct(blocks, nt);
}
int MPI_Type_create_hindexed(int count, const int blocklens[], const MPI_Aint displs[], MPI_Datatype old,
                             MPI_Datatype *nt) WEAK(MPI_Type_create_hindexed);

int PMPI_Type_create_struct(int count, const int blocklens[], const MPI_Aint displs[], const MPI_Datatype types[],
                            MPI_Datatype *nt) {
    if (count < 0) return MPI_ERR_COUNT;
    std::vector<Block> blocks;
    for (int i = 0; i < count; ++i) {
        if (!dtype_valid(types[i])) return MPI_ERR_TYPE;
        blocks.push_back(Block{(long)displs[i], blocklens[i], types[i]});
    }
    return make_struct(blocks, nt, true);
}
int MPI_Type_create_struct(int count, const int blocklens[], const MPI_Aint displs[], const MPI_Datatype types[],
                           MPI_Datatype *nt) WEAK(MPI_Type_create_struct);

int PMPI_Type_create_resized(MPI_Datatype old, MPI_Aint lb, MPI_Aint extent, MPI_Datatype *nt) {
    std::vector<Block> one{Block{0, 1, old}};
    if (!dtype_valid(old)) return MPI_ERR_TYPE;
    std::lock_guard<std::recursive_mutex> lk(g_mu);
    int rc = make_struct(one, nt);
    if (rc) return rc;
    Derived *d = derived(*nt);
    d->lb = (long)lb;
    d->extent = (long)extent;
    return MPI_SUCCESS;
}
int MPI_Type_create_resized(MPI_Datatype old, MPI_Aint lb, MPI_Aint extent, MPI_Datatype *nt) WEAK(MPI_Type_create_resized);

int PMPI_Type_dup(MPI_Datatype old, MPI_Datatype *nt) {
    long lb = 0, ext = 0;
    if (!type_bounds(old, lb, ext)) return MPI_ERR_TYPE;
    const int rc = PMPI_Type_create_resized(old, lb, ext, nt);
    // the copy has the committed state of the original, a builtin's copy is committed (MPI-3.1 §4.1.10)
    if (!rc) derived(*nt)->committed = dtype_committed(old);
    return rc;
}
int MPI_Type_dup(MPI_Datatype old, MPI_Datatype *nt) WEAK(MPI_Type_dup);

// Subarray (MPI-3.1 §4.1.3; the reference builds it from nested vectors,
// create_subarray.c / dataloop pack_subarray kernel pack_unpack.cu:256):
// one block per row of the fastest-varying dimension, then lb = 0 and
// extent = prod(sizes) * extent(old).
int PMPI_Type_create_subarray(int ndims, const int sizes[], const int subsizes[], const int starts[], int order,
                              MPI_Datatype old, MPI_Datatype *nt) {
    if (ndims <= 0) return MPI_ERR_DIMS;
    if (order != MPI_ORDER_C && order != MPI_ORDER_FORTRAN) return MPI_ERR_ARG;
    long olb = 0, oext = 0;
    if (!type_bounds(old, olb, oext)) return MPI_ERR_TYPE;
    std::vector<int> dim(ndims);  // dim[0] slowest ... dim[ndims-1] fastest
    for (int i = 0; i < ndims; ++i) {
        dim[i] = order == MPI_ORDER_C ? i : ndims - 1 - i;
        const int k = dim[i];
        if (sizes[k] <= 0 || subsizes[k] < 0 || starts[k] < 0 || starts[k] + subsizes[k] > sizes[k])
            return MPI_ERR_ARG;
    }
    std::vector<long> elem_stride(ndims);
    long total = 1;
    for (int i = ndims - 1; i >= 0; --i) {
        elem_stride[i] = total;
        total *= sizes[dim[i]];
    }
    const int fast = dim[ndims - 1];
    std::vector<Block> blocks;
    long nrows = 1;
    for (int i = 0; i + 1 < ndims; ++i) nrows *= subsizes[dim[i]];
    if (subsizes[fast] > 0)
        for (long r = 0; r < nrows; ++r) {
            long rem = r, e = starts[fast];
            for (int i = ndims - 2; i >= 0; --i) {
                const int k = dim[i];
                e += (starts[k] + rem % subsizes[k]) * elem_stride[i];
                rem /= subsizes[k];
            }
            blocks.push_back(Block{e * oext, subsizes[fast], old});
        }
    std::lock_guard<std::recursive_mutex> lk(g_mu);
    int rc = make_struct(blocks, nt);
    if (rc) return rc;
    Derived *d = derived(*nt);
    d->lb = 0;
    d->extent = total * oext;
    return MPI_SUCCESS;
}
int MPI_Type_create_subarray(int ndims, const int sizes[], const int subsizes[], const int starts[], int order,
                             MPI_Datatype old, MPI_Datatype *nt) WEAK(MPI_Type_create_subarray);

int PMPI_Type_commit(MPI_Datatype *dt) {
    std::lock_guard<std::recursive_mutex> lk(g_mu);
    if (dtype_is_builtin(*dt)) return MPI_SUCCESS;
    Derived *d = derived(*dt);
    if (!d) return MPI_ERR_TYPE;
    d->committed = true;
    return MPI_SUCCESS;
}
int MPI_Type_commit(MPI_Datatype *dt) WEAK(MPI_Type_commit);

int PMPI_Type_free(MPI_Datatype *dt) {
    std::lock_guard<std::recursive_mutex> lk(g_mu);
    Derived *d = derived(*dt);
    if (!d) return MPI_ERR_TYPE;
    d->live = false;
    d->segs.clear();
    *dt = MPI_DATATYPE_NULL;
    return MPI_SUCCESS;
}
int MPI_Type_free(MPI_Datatype *dt) WEAK(MPI_Type_free);

int PMPI_Pack_size(int incount, MPI_Datatype dt, MPI_Comm, int *size) {
    long s = dtype_size(dt);
    if (s < 0) return MPI_ERR_TYPE;
    *size = (int)(s * incount);
    return MPI_SUCCESS;
}
int MPI_Pack_size(int incount, MPI_Datatype dt, MPI_Comm comm, int *size) WEAK(MPI_Pack_size);

// Argument checks in pack.c:207-276's order: communicator, counts, null output buffer or
// position (MPI_ERR_ARG), datatype valid and committed, then a packed size that does not fit
// in outsize - *position: MPI_ERR_ARG (**argpackbuf), not MPI_ERR_TRUNCATE
int PMPI_Pack(const void *inbuf, int incount, MPI_Datatype dt, void *outbuf, int outsize, int *position,
              MPI_Comm comm) {
    std::lock_guard<std::recursive_mutex> lk(g_mu);
    if (comm != MPI_COMM_WORLD && comm != MPI_COMM_SELF) return MPI_ERR_COMM;
    if (incount < 0 || outsize < 0) return MPI_ERR_COUNT;
    if ((incount > 0 && !outbuf) || !position) return MPI_ERR_ARG;
    if (!dtype_valid(dt) || !dtype_committed(dt)) return MPI_ERR_TYPE;
    const long s = dtype_size(dt);
    if (*position < 0 || s * incount > (long)outsize - *position) return MPI_ERR_ARG;
    if (incount == 0) return MPI_SUCCESS;
    int rc = pack_impl((const char *)inbuf, incount, dt, (char *)outbuf + *position, false);
    if (!rc) *position += (int)(s * incount);
    return rc;
}
int MPI_Pack(const void *inbuf, int incount, MPI_Datatype dt, void *outbuf, int outsize, int *position, MPI_Comm comm) WEAK(MPI_Pack);

// Argument checks of unpack.c:207-229: null input buffer (MPI_ERR_ARG), counts, communicator,
// datatype valid and committed.  The reference does not check the packed size against insize
// (its unpack reads past the buffer); here that is MPI_ERR_TRUNCATE.
int PMPI_Unpack(const void *inbuf, int insize, int *position, void *outbuf, int outcount, MPI_Datatype dt,
                MPI_Comm comm) {
    std::lock_guard<std::recursive_mutex> lk(g_mu);
    if ((insize > 0 && !inbuf) || !position) return MPI_ERR_ARG;
    if (insize < 0 || outcount < 0) return MPI_ERR_COUNT;
    if (comm != MPI_COMM_WORLD && comm != MPI_COMM_SELF) return MPI_ERR_COMM;
    if (!dtype_valid(dt) || !dtype_committed(dt)) return MPI_ERR_TYPE;
    const long s = dtype_size(dt);
    if (*position < 0 || *position + s * outcount > insize) return MPI_ERR_TRUNCATE;
    if (outcount == 0) return MPI_SUCCESS;
    int rc = pack_impl((const char *)inbuf + *position, outcount, dt, (char *)outbuf, true);
    if (!rc) *position += (int)(s * outcount);
    return rc;
}
int MPI_Unpack(const void *inbuf, int insize, int *position, void *outbuf, int outcount, MPI_Datatype dt, MPI_Comm comm) WEAK(MPI_Unpack);

}  // extern "C"
