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
// pack_unpack_vector_kernel paths (pack_unpack.cu:419).  Host buffers are
// copied on the host, as the reference does for host memory.
#include "datatype.h"

#include <string.h>

#include <mutex>
#include <vector>

#include "../../../include/mv2h.h"
#include "../common.h"

namespace {

struct Seg {
    long off, len;
};

struct Derived {
    bool live = false, committed = false;
    long size = 0, lb = 0, extent = 0, true_lb = 0, true_extent = 0;
    std::vector<Seg> segs;  // one element, sorted by construction order, merged
};

std::vector<Derived> g_types;
std::recursive_mutex g_mu;
constexpr int kDerivedBase = (int)0x8c000010;

Derived *derived(MPI_Datatype dt) {
    const unsigned idx = (unsigned)(dt - kDerivedBase);
    if ((dt & 0xfc000000) != (int)0x8c000000 || idx >= g_types.size() || !g_types[idx].live) return nullptr;
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

int make_type(const std::vector<long> &block_offsets, int blocklen, MPI_Datatype old, MPI_Datatype *out) {
    std::lock_guard<std::recursive_mutex> lk(g_mu);
    std::vector<Seg> os;
    long oext = 0, osize = 0;
    if (!type_segs(old, os, oext, osize)) return MPI_ERR_TYPE;
    if (blocklen < 0) return MPI_ERR_ARG;
    Derived d;
    d.live = true;
    long lo = 0, hi = 0;
    bool first = true;
    for (long bo : block_offsets) {
        for (int k = 0; k < blocklen; ++k) {
            for (const Seg &s : os) {
                const Seg t{bo + (long)k * oext + s.off, s.len};
                push_merge(d.segs, t);
                if (first || t.off < lo) lo = t.off;
                if (first || t.off + t.len > hi) hi = t.off + t.len;
                first = false;
            }
        }
    }
    d.size = (long)block_offsets.size() * blocklen * osize;
    d.true_lb = first ? 0 : lo;
    d.true_extent = first ? 0 : hi - lo;
    // extent per MPI: lb = min block start, ub = max block end (old extent granularity)
    long lb = 0, ub = 0;
    first = true;
    for (long bo : block_offsets) {
        const long b0 = bo, b1 = bo + (long)blocklen * oext;
        if (first || b0 < lb) lb = b0;
        if (first || b1 > ub) ub = b1;
        first = false;
    }
    d.lb = first ? 0 : lb;
    d.extent = first ? 0 : ub - lb;
    g_types.push_back(d);
    *out = kDerivedBase + (int)(g_types.size() - 1);
    return MPI_SUCCESS;
}

// regular layout of `count` elements: nblocks x blk bytes at constant stride
bool regular(const Derived *d, long extent, int count, long &nblocks, long &blk, long &stride) {
    const auto &s = d->segs;
    if (s.empty()) return false;
    blk = s[0].len;
    stride = s.size() > 1 ? s[1].off - s[0].off : extent;
    if (s[0].off != 0) return false;
    for (size_t i = 0; i < s.size(); ++i)
        if (s[i].len != blk || s[i].off != (long)i * stride) return false;
    if (count > 1 && (long)s.size() * stride != extent) return false;
    nblocks = (long)s.size() * count;
    return stride >= blk;
}

int pack_impl(const char *in, int count, MPI_Datatype dt, char *out, bool unpack) {
    std::vector<Seg> segs;
    long ext = 0, size = 0;
    if (!type_segs(dt, segs, ext, size)) return MPI_ERR_TYPE;
    const bool din = mv2h_is_device_ptr(in), dout = mv2h_is_device_ptr(out);
    Derived *d = derived(dt);
    if (!din && !dout) {
        // host <-> host: reference semantics, host copies
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
        void *tmp = nullptr;
        if (!unpack) {
            // pack: src strided, dst packed
            if (!din) {
                if (mv2h_malloc(&tmp, span)) return MPI_ERR_NO_MEM;
                mv2h_memcpy_htod(tmp, in, span);
                int rc = pack_impl((const char *)tmp, count, dt, out, false);
                mv2h_free(tmp);
                return rc;
            }
            if (mv2h_malloc(&tmp, packed)) return MPI_ERR_NO_MEM;
            int rc = pack_impl(in, count, dt, (char *)tmp, false);
            if (!rc) mv2h_memcpy_dtoh(out, tmp, packed);
            mv2h_free(tmp);
            return rc;
        }
        if (!din) {
            if (mv2h_malloc(&tmp, packed)) return MPI_ERR_NO_MEM;
            mv2h_memcpy_htod(tmp, in, packed);
            int rc = pack_impl((const char *)tmp, count, dt, out, true);
            mv2h_free(tmp);
            return rc;
        }
        // unpack into a host destination: copy its current bytes so gaps survive
        if (mv2h_malloc(&tmp, span)) return MPI_ERR_NO_MEM;
        mv2h_memcpy_htod(tmp, out, span);
        int rc = pack_impl(in, count, dt, (char *)tmp, true);
        if (!rc) mv2h_memcpy_dtoh(out, tmp, span);
        mv2h_free(tmp);
        return rc;
    }
    // device <-> device
    long nb = 0, blk = 0, stride = 0;
    if (d && regular(d, ext, count, nb, blk, stride)) {
        int rc = unpack ? mv2h_unpack_strided(in, out, nb, blk, stride, nullptr)
                        : mv2h_pack_strided(in, out, nb, blk, stride, nullptr);
        return rc ? MPI_ERR_OTHER : MPI_SUCCESS;
    }
    if (d && count > 1 && regular(d, ext, 1, nb, blk, stride)) {
        long pos = 0;
        for (int e = 0; e < count; ++e) {
            int rc = unpack ? mv2h_unpack_strided(in + pos, out + (long)e * ext, nb, blk, stride, nullptr)
                            : mv2h_pack_strided(in + (long)e * ext, out + pos, nb, blk, stride, nullptr);
            if (rc) return MPI_ERR_OTHER;
            pos += size;
        }
        return MPI_SUCCESS;
    }
    // irregular layouts: one device copy per segment
    long pos = 0;
    for (int e = 0; e < count; ++e)
        for (const Seg &s : segs) {
            int rc = unpack ? mv2h_memcpy_dtod(out + (long)e * ext + s.off, in + pos, s.len)
                            : mv2h_memcpy_dtod(out + pos, in + (long)e * ext + s.off, s.len);
            if (rc) return MPI_ERR_OTHER;
            pos += s.len;
        }
    return MPI_SUCCESS;
}

}  // namespace

bool dtype_valid(MPI_Datatype dt) { return mv2::dtype_lookup(dt) != nullptr || derived(dt) != nullptr; }
bool dtype_is_builtin(MPI_Datatype dt) { return mv2::dtype_lookup(dt) != nullptr; }
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
long dtype_span(MPI_Datatype dt, int count) {
    if (count <= 0) return 0;
    if (const mv2::DtypeInfo *b = mv2::dtype_lookup(dt)) return (long)count * b->extent;
    Derived *d = derived(dt);
    if (!d) return -1;
    return (long)(count - 1) * d->extent + d->true_lb + d->true_extent;
}

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
    if (stride < 0) return MPI_ERR_ARG;  // negative strides: not supported yet
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
    for (int i = 0; i < count; ++i) {
        if (displs[i] < 0) return MPI_ERR_ARG;
        offs.push_back((long)displs[i] * ext);
    }
    return make_type(offs, blocklen, old, nt);
}
int MPI_Type_create_indexed_block(int count, int blocklen, const int displs[], MPI_Datatype old, MPI_Datatype *nt) WEAK(MPI_Type_create_indexed_block);

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

int PMPI_Pack(const void *inbuf, int incount, MPI_Datatype dt, void *outbuf, int outsize, int *position, MPI_Comm) {
    std::lock_guard<std::recursive_mutex> lk(g_mu);
    if (incount < 0) return MPI_ERR_COUNT;
    const long s = dtype_size(dt);
    if (s < 0) return MPI_ERR_TYPE;
    if (*position + s * incount > outsize) return MPI_ERR_TRUNCATE;
    if (incount == 0) return MPI_SUCCESS;
    int rc = pack_impl((const char *)inbuf, incount, dt, (char *)outbuf + *position, false);
    if (!rc) *position += (int)(s * incount);
    return rc;
}
int MPI_Pack(const void *inbuf, int incount, MPI_Datatype dt, void *outbuf, int outsize, int *position, MPI_Comm comm) WEAK(MPI_Pack);

int PMPI_Unpack(const void *inbuf, int insize, int *position, void *outbuf, int outcount, MPI_Datatype dt, MPI_Comm) {
    std::lock_guard<std::recursive_mutex> lk(g_mu);
    if (outcount < 0) return MPI_ERR_COUNT;
    const long s = dtype_size(dt);
    if (s < 0) return MPI_ERR_TYPE;
    if (*position + s * outcount > insize) return MPI_ERR_TRUNCATE;
    if (outcount == 0) return MPI_SUCCESS;
    int rc = pack_impl((const char *)inbuf + *position, outcount, dt, (char *)outbuf, true);
    if (!rc) *position += (int)(s * outcount);
    return rc;
}
int MPI_Unpack(const void *inbuf, int insize, int *position, void *outbuf, int outcount, MPI_Datatype dt, MPI_Comm comm) WEAK(MPI_Unpack);

}  // extern "C"
