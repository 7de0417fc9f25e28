// mpit.cpp — the MPI_T tool information interface over the collective hot
// path.  Performance variables: per-algorithm call counters and timers under
// the reference's names and categories (runtime/pvars.h; registered in the
// reference by src/mpi_t/mv2_mpit.c with READONLY | SUM flags: not
// continuous, started and stopped per handle, never written or reset).
// Control variables: the MV2_* selection knobs this path honours
// (runtime/orders.h Knobs), read-only, under their environment names.
// Semantics follow MPICH's src/mpi_t/*.c (name/len convention, error codes,
// MPI_T_PVAR_ALL_HANDLES, the start offset of a SUM variable).
#include <stdint.h>
#include <string.h>

#include <mutex>
#include <string>
#include <vector>

#include "../../../include/mpi.h"
#include "../runtime/orders.h"
#include "../runtime/pvars.h"

using namespace mv2;

struct MPIR_T_pvar_handle_s {
    int index;     // pvar index
    bool started;
    double accum;  // value collected while started (counters as double: exact below 2^53)
    double offset; // variable's value when last started
    MPIR_T_pvar_session_s *session;
};
struct MPIR_T_pvar_session_s {
    std::vector<MPIR_T_pvar_handle_s *> handles;
};
struct MPIR_T_cvar_handle_s {
    int index;
};
struct MPIR_T_enum_s {
    int unused;
};

extern "C" {
static MPIR_T_pvar_handle_s g_all_handles_tag{};
MPIR_T_pvar_handle_s *const MPI_T_PVAR_ALL_HANDLES = &g_all_handles_tag;
}

namespace {

std::recursive_mutex g_mu;
int g_init = 0;

// ---- performance variables: counters [0, PV_COUNT), then the timers ----
struct PvarRef {
    int id;
    bool timer;
};
const std::vector<PvarRef> &pvars() {
    static const std::vector<PvarRef> v = [] {
        std::vector<PvarRef> r;
        for (int i = 0; i < PV_COUNT; ++i) r.push_back({i, false});
        for (int i = 0; i < PV_COUNT; ++i)
            if (pvar_desc(i).timer) r.push_back({i, true});
        return r;
    }();
    return v;
}
double pvar_value(int index) {
    const PvarRef &r = pvars()[(size_t)index];
    return r.timer ? pvar_seconds(r.id) : (double)pvar_count(r.id);
}

// ---- control variables: the selection knobs (orders.h Knobs) ----
struct CvarDesc {
    const char *name;
    size_t off;
    bool wide;  // int64 (MPI_LONG_LONG) else int32 (MPI_INT)
    const char *desc;
};
#define KN(f) offsetof(Knobs, f)
const CvarDesc kCvars[] = {
    {"MV2_USE_SHARED_MEM", KN(enable_shmem_collectives), false, "shared-memory collectives (ch3_shmem_coll.c)"},
    {"MV2_USE_SHMEM_ALLREDUCE", KN(enable_shmem_allreduce), false, "two-level shmem allreduce"},
    {"MV2_USE_SHMEM_REDUCE", KN(enable_shmem_reduce), false, "two-level shmem reduce"},
    {"MV2_ENABLE_SKIP_TUNING_TABLE_SEARCH", KN(enable_skip_search), false, "skip the tuning tables for small messages"},
    {"MV2_COLL_SKIP_TABLE_THRESHOLD", KN(coll_skip_thr), false, "small-message threshold of the skip (bytes)"},
    {"MV2_ENABLE_ALLREDUCE_SKIP_SMALL_MESSAGE_TUNING_TABLE_SEARCH", KN(allred_skip_small), false,
     "allreduce small-message shortcuts"},
    {"MV2_ENABLE_ALLREDUCE_SKIP_LARGE_MESSAGE_TUNING_TABLE_SEARCH", KN(allred_skip_large), false,
     "allreduce large-message shortcut (ring)"},
    {"MV2_ENABLE_TOPO_AWARE_COLLECTIVES", KN(enable_topo), false, "topology-aware collectives"},
    {"MV2_USE_TOPO_AWARE_ALLREDUCE", KN(use_topo_allreduce), false, "topology-aware allreduce"},
    {"MV2_TOPO_AWARE_ALLREDUCE_MIN_MSG", KN(topo_allred_min), false, "topology-aware allreduce from (bytes)"},
    {"MV2_TOPO_AWARE_ALLREDUCE_MAX_MSG", KN(topo_allred_max), false, "topology-aware allreduce up to (bytes)"},
    {"MV2_USE_TOPO_AWARE_REDUCE", KN(use_topo_reduce), false, "topology-aware reduce"},
    {"MV2_TOPO_AWARE_REDUCE_MIN_MSG", KN(topo_red_min), false, "topology-aware reduce from (bytes)"},
    {"MV2_TOPO_AWARE_REDUCE_MAX_MSG", KN(topo_red_max), false, "topology-aware reduce up to (bytes)"},
    {"MV2_TOPO_AWARE_REDUCE_PPN_THRESHOLD", KN(topo_red_ppn), false, "topology-aware reduce ppn threshold"},
    {"MV2_TOPO_AWARE_REDUCE_NODE_THRESHOLD", KN(topo_red_nodes), false, "topology-aware reduce node threshold"},
    {"MV2_SHMEM_REDUCE_TREE_DEGREE", KN(tree_degree), false, "degree of the shm reduce tree"},
    {"MV2_ALLRED_USE_RING", KN(allred_use_ring), false, "ring allreduce for large messages"},
    {"MV2_ALLREDUCE_RING_ALGO_THRESHOLD", KN(allred_ring_thr), true, "ring allreduce from (bytes)"},
    {"MV2_ALLREDUCE_RING_ALGO_PPN_THRESHOLD", KN(allred_ring_ppn), false, "ring allreduce up to this many ranks per node"},
    {"MV2_SMP_USE_CMA", KN(smp_use_cma), false, "CMA (selects the CMA reduce tables)"},
    {"MV2_USE_KNOMIAL_REDUCE", KN(use_knomial_reduce), false, "knomial intra-node reduce"},
    {"MV2_USE_INTER_KNOMIAL_REDUCE_FACTOR", KN(reduce_inter_k), false, "knomial reduce factor (-1: table)"},
    {"MV2_SHMEM_COLL_MAX_MSG_SIZE", KN(shmem_coll_max_msg), false, "shmem collective slot size (bytes)"},
    {"MV2_INTRA_SHMEM_REDUCE_MSG", KN(shmem_intra_reduce_msg), false, "shmem reduce up to (bytes)"},
    {"MV2_RED_SCAT_RING_ALGO_THRESHOLD", KN(red_scat_ring_thr), true, "ring reduce_scatter from (bytes)"},
};
#undef KN
constexpr int kNumCvars = (int)(sizeof(kCvars) / sizeof(kCvars[0]));

// ---- categories ----
struct Cat {
    const char *name, *desc;
};
const Cat kCats[] = {
    {"Allreduce Algorithms", "MV2 allreduce algorithm calls and time"},
    {"Reduce Algorithms", "MV2 reduce algorithm calls and time"},
    {"Reduce_scatter Algorithms", "MV2 reduce_scatter algorithm calls and time"},
    {"Shmem Collective Calls", "MV2 shared-memory collective calls"},
    {"Collective Selection", "MV2_* variables that move the collective algorithm selection"},
};
constexpr int kNumCats = (int)(sizeof(kCats) / sizeof(kCats[0]));

std::vector<int> cat_pvars(int c) {
    std::vector<int> v;
    const auto &pv = pvars();
    for (size_t i = 0; i < pv.size(); ++i)
        if (c < kNumCats - 1 && !strcmp(pvar_desc(pv[i].id).category, kCats[c].name)) v.push_back((int)i);
    return v;
}

// MPI-3.1 §14.3.3: copy up to *len - 1 characters; *len returns strlen + 1
void put_str(const char *src, char *dst, int *len) {
    if (!len) return;
    const int need = (int)strlen(src) + 1;
    if (dst && *len > 0) {
        const int n = need < *len ? need : *len;
        memcpy(dst, src, (size_t)n - 1);
        dst[n - 1] = '\0';
    }
    *len = need;
}

std::string pvar_name(int index) {
    const PvarRef &r = pvars()[(size_t)index];
    return r.timer ? pvar_desc(r.id).timer : pvar_desc(r.id).counter;
}

}  // namespace

#define WEAK(name) __attribute__((weak, alias("P" #name)))
#define REQUIRE_INIT()                                 \
    std::lock_guard<std::recursive_mutex> lk(g_mu);    \
    if (g_init <= 0) return MPI_T_ERR_NOT_INITIALIZED

extern "C" {

int PMPI_T_init_thread(int required, int *provided) {
    std::lock_guard<std::recursive_mutex> lk(g_mu);
    (void)required;
    ++g_init;
    if (provided) *provided = MPI_THREAD_MULTIPLE;  // every entry takes the interface's lock
    return MPI_SUCCESS;
}
int PMPI_T_finalize(void) {
    REQUIRE_INIT();
    --g_init;
    return MPI_SUCCESS;
}

// no enumerations are exported
int PMPI_T_enum_get_info(MPI_T_enum, int *, char *, int *) {
    REQUIRE_INIT();
    return MPI_T_ERR_INVALID_HANDLE;
}
int PMPI_T_enum_get_item(MPI_T_enum, int, int *, char *, int *) {
    REQUIRE_INIT();
    return MPI_T_ERR_INVALID_HANDLE;
}

// ---- cvars ----
int PMPI_T_cvar_get_num(int *num) {
    REQUIRE_INIT();
    if (!num) return MPI_ERR_ARG;
    *num = kNumCvars;
    return MPI_SUCCESS;
}
int PMPI_T_cvar_get_info(int i, char *name, int *name_len, int *verbosity, MPI_Datatype *datatype,
                         MPI_T_enum *enumtype, char *desc, int *desc_len, int *binding, int *scope) {
    REQUIRE_INIT();
    if (i < 0 || i >= kNumCvars) return MPI_T_ERR_INVALID_INDEX;
    put_str(kCvars[i].name, name, name_len);
    put_str(kCvars[i].desc, desc, desc_len);
    if (verbosity) *verbosity = MPI_T_VERBOSITY_TUNER_BASIC;
    if (datatype) *datatype = kCvars[i].wide ? MPI_LONG_LONG : MPI_INT;
    if (enumtype) *enumtype = MPI_T_ENUM_NULL;
    if (binding) *binding = MPI_T_BIND_NO_OBJECT;
    if (scope) *scope = MPI_T_SCOPE_ALL_EQ;  // every rank must see the same value (checked at MPI_Init)
    return MPI_SUCCESS;
}
int PMPI_T_cvar_get_index(const char *name, int *index) {
    REQUIRE_INIT();
    if (!name || !index) return MPI_ERR_ARG;
    for (int i = 0; i < kNumCvars; ++i)
        if (!strcmp(name, kCvars[i].name)) {
            *index = i;
            return MPI_SUCCESS;
        }
    return MPI_T_ERR_INVALID_NAME;
}
int PMPI_T_cvar_handle_alloc(int i, void *, MPI_T_cvar_handle *handle, int *count) {
    REQUIRE_INIT();
    if (i < 0 || i >= kNumCvars) return MPI_T_ERR_INVALID_INDEX;
    if (!handle || !count) return MPI_ERR_ARG;
    *handle = new MPIR_T_cvar_handle_s{i};
    *count = 1;
    return MPI_SUCCESS;
}
int PMPI_T_cvar_handle_free(MPI_T_cvar_handle *handle) {
    REQUIRE_INIT();
    if (!handle || !*handle) return MPI_T_ERR_INVALID_HANDLE;
    delete *handle;
    *handle = MPI_T_CVAR_HANDLE_NULL;
    return MPI_SUCCESS;
}
int PMPI_T_cvar_read(MPI_T_cvar_handle handle, void *buf) {
    REQUIRE_INIT();
    if (!handle) return MPI_T_ERR_INVALID_HANDLE;
    if (!buf) return MPI_ERR_ARG;
    const CvarDesc &c = kCvars[handle->index];
    const char *k = (const char *)&knobs() + c.off;
    if (c.wide) {
        long long v;
        int64_t x;
        memcpy(&x, k, sizeof(x));
        v = (long long)x;
        memcpy(buf, &v, sizeof(v));
    } else {
        int v;
        int32_t x;
        memcpy(&x, k, sizeof(x));
        v = (int)x;
        memcpy(buf, &v, sizeof(v));
    }
    return MPI_SUCCESS;
}
// the selection must be identical on every rank and is fixed at MPI_Init (the
// environment is the way to set it)
int PMPI_T_cvar_write(MPI_T_cvar_handle handle, const void *) {
    REQUIRE_INIT();
    if (!handle) return MPI_T_ERR_INVALID_HANDLE;
    return MPI_T_ERR_CVAR_SET_NEVER;
}

// ---- pvars ----
int PMPI_T_pvar_get_num(int *num) {
    REQUIRE_INIT();
    if (!num) return MPI_ERR_ARG;
    *num = (int)pvars().size();
    return MPI_SUCCESS;
}
int PMPI_T_pvar_get_info(int i, char *name, int *name_len, int *verbosity, int *var_class, MPI_Datatype *datatype,
                         MPI_T_enum *enumtype, char *desc, int *desc_len, int *binding, int *readonly,
                         int *continuous, int *atomic) {
    REQUIRE_INIT();
    if (i < 0 || i >= (int)pvars().size()) return MPI_T_ERR_INVALID_INDEX;
    const PvarRef &r = pvars()[(size_t)i];
    put_str(pvar_name(i).c_str(), name, name_len);
    const std::string d = r.timer ? std::string("Time spent in the algorithm counted by ") + pvar_desc(r.id).counter
                                  : std::string(pvar_desc(r.id).desc);
    put_str(d.c_str(), desc, desc_len);
    if (verbosity) *verbosity = MPI_T_VERBOSITY_USER_BASIC;
    if (var_class) *var_class = r.timer ? MPI_T_PVAR_CLASS_TIMER : MPI_T_PVAR_CLASS_COUNTER;
    if (datatype) *datatype = r.timer ? MPI_DOUBLE : MPI_UNSIGNED_LONG_LONG;
    if (enumtype) *enumtype = MPI_T_ENUM_NULL;
    if (binding) *binding = MPI_T_BIND_NO_OBJECT;
    if (readonly) *readonly = 1;
    if (continuous) *continuous = 0;
    if (atomic) *atomic = 0;
    return MPI_SUCCESS;
}
int PMPI_T_pvar_get_index(const char *name, int var_class, int *index) {
    REQUIRE_INIT();
    if (!name || !index) return MPI_ERR_ARG;
    for (int i = 0; i < (int)pvars().size(); ++i) {
        const int cls = pvars()[(size_t)i].timer ? MPI_T_PVAR_CLASS_TIMER : MPI_T_PVAR_CLASS_COUNTER;
        if (cls == var_class && pvar_name(i) == name) {
            *index = i;
            return MPI_SUCCESS;
        }
    }
    return MPI_T_ERR_INVALID_NAME;
}
int PMPI_T_pvar_session_create(MPI_T_pvar_session *session) {
    REQUIRE_INIT();
    if (!session) return MPI_ERR_ARG;
    *session = new MPIR_T_pvar_session_s();
    return MPI_SUCCESS;
}
int PMPI_T_pvar_session_free(MPI_T_pvar_session *session) {
    REQUIRE_INIT();
    if (!session || !*session) return MPI_T_ERR_INVALID_SESSION;
    for (auto *h : (*session)->handles) delete h;
    delete *session;
    *session = MPI_T_PVAR_SESSION_NULL;
    return MPI_SUCCESS;
}
int PMPI_T_pvar_handle_alloc(MPI_T_pvar_session session, int i, void *, MPI_T_pvar_handle *handle, int *count) {
    REQUIRE_INIT();
    if (!session) return MPI_T_ERR_INVALID_SESSION;
    if (i < 0 || i >= (int)pvars().size()) return MPI_T_ERR_INVALID_INDEX;
    if (!handle || !count) return MPI_ERR_ARG;
    auto *h = new MPIR_T_pvar_handle_s{i, false, 0.0, 0.0, session};
    session->handles.push_back(h);
    *handle = h;
    *count = 1;
    return MPI_SUCCESS;
}
int PMPI_T_pvar_handle_free(MPI_T_pvar_session session, MPI_T_pvar_handle *handle) {
    REQUIRE_INIT();
    if (!session) return MPI_T_ERR_INVALID_SESSION;
    if (!handle || !*handle || *handle == MPI_T_PVAR_ALL_HANDLES || (*handle)->session != session)
        return MPI_T_ERR_INVALID_HANDLE;
    auto &v = session->handles;
    for (size_t k = 0; k < v.size(); ++k)
        if (v[k] == *handle) {
            v.erase(v.begin() + (long)k);
            break;
        }
    delete *handle;
    *handle = MPI_T_PVAR_HANDLE_NULL;
    return MPI_SUCCESS;
}

static int each_handle(MPI_T_pvar_session session, MPI_T_pvar_handle handle, void (*fn)(MPIR_T_pvar_handle_s *)) {
    if (!session) return MPI_T_ERR_INVALID_SESSION;
    if (handle == MPI_T_PVAR_ALL_HANDLES) {
        for (auto *h : session->handles) fn(h);
        return MPI_SUCCESS;
    }
    if (!handle || handle->session != session) return MPI_T_ERR_INVALID_HANDLE;
    fn(handle);
    return MPI_SUCCESS;
}
int PMPI_T_pvar_start(MPI_T_pvar_session session, MPI_T_pvar_handle handle) {
    REQUIRE_INIT();
    return each_handle(session, handle, [](MPIR_T_pvar_handle_s *h) {
        if (h->started) return;
        h->offset = pvar_value(h->index);
        h->started = true;
    });
}
int PMPI_T_pvar_stop(MPI_T_pvar_session session, MPI_T_pvar_handle handle) {
    REQUIRE_INIT();
    return each_handle(session, handle, [](MPIR_T_pvar_handle_s *h) {
        if (!h->started) return;
        h->accum += pvar_value(h->index) - h->offset;
        h->started = false;
    });
}
int PMPI_T_pvar_read(MPI_T_pvar_session session, MPI_T_pvar_handle handle, void *buf) {
    REQUIRE_INIT();
    if (!session) return MPI_T_ERR_INVALID_SESSION;
    if (handle == MPI_T_PVAR_ALL_HANDLES || !handle || handle->session != session) return MPI_T_ERR_INVALID_HANDLE;
    if (!buf) return MPI_ERR_ARG;
    const double v = handle->accum + (handle->started ? pvar_value(handle->index) - handle->offset : 0.0);
    if (pvars()[(size_t)handle->index].timer) {
        memcpy(buf, &v, sizeof(v));
    } else {
        const unsigned long long c = (unsigned long long)(v + 0.5);
        memcpy(buf, &c, sizeof(c));
    }
    return MPI_SUCCESS;
}
// READONLY variables (mv2_mpit.c registers them MPIR_T_PVAR_FLAG_READONLY)
int PMPI_T_pvar_write(MPI_T_pvar_session session, MPI_T_pvar_handle handle, const void *) {
    REQUIRE_INIT();
    if (!session) return MPI_T_ERR_INVALID_SESSION;
    if (!handle || (handle != MPI_T_PVAR_ALL_HANDLES && handle->session != session)) return MPI_T_ERR_INVALID_HANDLE;
    return MPI_T_ERR_PVAR_NO_WRITE;
}
int PMPI_T_pvar_reset(MPI_T_pvar_session session, MPI_T_pvar_handle handle) {
    return PMPI_T_pvar_write(session, handle, nullptr);
}
int PMPI_T_pvar_readreset(MPI_T_pvar_session session, MPI_T_pvar_handle handle, void *) {
    return PMPI_T_pvar_write(session, handle, nullptr);
}

// ---- categories ----
int PMPI_T_category_get_num(int *num) {
    REQUIRE_INIT();
    if (!num) return MPI_ERR_ARG;
    *num = kNumCats;
    return MPI_SUCCESS;
}
int PMPI_T_category_get_info(int c, char *name, int *name_len, char *desc, int *desc_len, int *num_cvars,
                             int *num_pvars, int *num_categories) {
    REQUIRE_INIT();
    if (c < 0 || c >= kNumCats) return MPI_T_ERR_INVALID_INDEX;
    put_str(kCats[c].name, name, name_len);
    put_str(kCats[c].desc, desc, desc_len);
    if (num_cvars) *num_cvars = c == kNumCats - 1 ? kNumCvars : 0;
    if (num_pvars) *num_pvars = (int)cat_pvars(c).size();
    if (num_categories) *num_categories = 0;
    return MPI_SUCCESS;
}
int PMPI_T_category_get_index(const char *name, int *index) {
    REQUIRE_INIT();
    if (!name || !index) return MPI_ERR_ARG;
    for (int c = 0; c < kNumCats; ++c)
        if (!strcmp(name, kCats[c].name)) {
            *index = c;
            return MPI_SUCCESS;
        }
    return MPI_T_ERR_INVALID_NAME;
}
int PMPI_T_category_get_cvars(int c, int len, int indices[]) {
    REQUIRE_INIT();
    if (c < 0 || c >= kNumCats) return MPI_T_ERR_INVALID_INDEX;
    if (c == kNumCats - 1)
        for (int i = 0; i < len && i < kNumCvars; ++i) indices[i] = i;
    return MPI_SUCCESS;
}
int PMPI_T_category_get_pvars(int c, int len, int indices[]) {
    REQUIRE_INIT();
    if (c < 0 || c >= kNumCats) return MPI_T_ERR_INVALID_INDEX;
    const std::vector<int> v = cat_pvars(c);
    for (int i = 0; i < len && i < (int)v.size(); ++i) indices[i] = v[(size_t)i];
    return MPI_SUCCESS;
}
int PMPI_T_category_get_categories(int c, int, int *) {
    REQUIRE_INIT();
    if (c < 0 || c >= kNumCats) return MPI_T_ERR_INVALID_INDEX;
    return MPI_SUCCESS;
}
int PMPI_T_category_changed(int *stamp) {
    REQUIRE_INIT();
    if (!stamp) return MPI_ERR_ARG;
    *stamp = 0;  // the variable set is static
    return MPI_SUCCESS;
}

int MPI_T_init_thread(int required, int *provided) WEAK(MPI_T_init_thread);
int MPI_T_finalize(void) WEAK(MPI_T_finalize);
int MPI_T_enum_get_info(MPI_T_enum e, int *num, char *name, int *len) WEAK(MPI_T_enum_get_info);
int MPI_T_enum_get_item(MPI_T_enum e, int i, int *v, char *name, int *len) WEAK(MPI_T_enum_get_item);
int MPI_T_cvar_get_num(int *num) WEAK(MPI_T_cvar_get_num);
int MPI_T_cvar_get_info(int i, char *name, int *nl, int *verb, MPI_Datatype *dt, MPI_T_enum *e, char *desc, int *dl,
                        int *bind, int *scope) WEAK(MPI_T_cvar_get_info);
int MPI_T_cvar_get_index(const char *name, int *i) WEAK(MPI_T_cvar_get_index);
int MPI_T_cvar_handle_alloc(int i, void *obj, MPI_T_cvar_handle *h, int *count) WEAK(MPI_T_cvar_handle_alloc);
int MPI_T_cvar_handle_free(MPI_T_cvar_handle *h) WEAK(MPI_T_cvar_handle_free);
int MPI_T_cvar_read(MPI_T_cvar_handle h, void *buf) WEAK(MPI_T_cvar_read);
int MPI_T_cvar_write(MPI_T_cvar_handle h, const void *buf) WEAK(MPI_T_cvar_write);
int MPI_T_pvar_get_num(int *num) WEAK(MPI_T_pvar_get_num);
int MPI_T_pvar_get_info(int i, char *name, int *nl, int *verb, int *cls, MPI_Datatype *dt, MPI_T_enum *e, char *desc,
                        int *dl, int *bind, int *ro, int *cont, int *atomic) WEAK(MPI_T_pvar_get_info);
int MPI_T_pvar_get_index(const char *name, int cls, int *i) WEAK(MPI_T_pvar_get_index);
int MPI_T_pvar_session_create(MPI_T_pvar_session *s) WEAK(MPI_T_pvar_session_create);
int MPI_T_pvar_session_free(MPI_T_pvar_session *s) WEAK(MPI_T_pvar_session_free);
int MPI_T_pvar_handle_alloc(MPI_T_pvar_session s, int i, void *obj, MPI_T_pvar_handle *h, int *count)
    WEAK(MPI_T_pvar_handle_alloc);
int MPI_T_pvar_handle_free(MPI_T_pvar_session s, MPI_T_pvar_handle *h) WEAK(MPI_T_pvar_handle_free);
int MPI_T_pvar_start(MPI_T_pvar_session s, MPI_T_pvar_handle h) WEAK(MPI_T_pvar_start);
int MPI_T_pvar_stop(MPI_T_pvar_session s, MPI_T_pvar_handle h) WEAK(MPI_T_pvar_stop);
int MPI_T_pvar_read(MPI_T_pvar_session s, MPI_T_pvar_handle h, void *buf) WEAK(MPI_T_pvar_read);
int MPI_T_pvar_write(MPI_T_pvar_session s, MPI_T_pvar_handle h, const void *buf) WEAK(MPI_T_pvar_write);
int MPI_T_pvar_reset(MPI_T_pvar_session s, MPI_T_pvar_handle h) WEAK(MPI_T_pvar_reset);
int MPI_T_pvar_readreset(MPI_T_pvar_session s, MPI_T_pvar_handle h, void *buf) WEAK(MPI_T_pvar_readreset);
int MPI_T_category_get_num(int *num) WEAK(MPI_T_category_get_num);
int MPI_T_category_get_info(int c, char *name, int *nl, char *desc, int *dl, int *nc, int *np, int *ncat)
    WEAK(MPI_T_category_get_info);
int MPI_T_category_get_index(const char *name, int *c) WEAK(MPI_T_category_get_index);
int MPI_T_category_get_cvars(int c, int len, int indices[]) WEAK(MPI_T_category_get_cvars);
int MPI_T_category_get_pvars(int c, int len, int indices[]) WEAK(MPI_T_category_get_pvars);
int MPI_T_category_get_categories(int c, int len, int indices[]) WEAK(MPI_T_category_get_categories);
int MPI_T_category_changed(int *stamp) WEAK(MPI_T_category_changed);

}  // extern "C"
