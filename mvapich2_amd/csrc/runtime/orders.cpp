// orders.cpp — one-node algorithm selection and reduction-order programs
// (see orders.h).  Each algorithm is restated as a symbolic run of its
// message schedule: every rank's partial result for every block is an
// expression tree whose internal nodes are uop(in, inout) calls, with the
// inout operand (the reference's accumulator) on the left.  compile() turns
// the final tree of each block into a Prog: each subtree's value lives in
// the register of its leftmost leaf, so a tree over distinct ranks needs no
// temporaries.
#include "orders.h"

#include <stdlib.h>
#include <string.h>

#include <vector>

#include "../common.h"

namespace mv2 {

// ---------------------------------------------------------------------------
// knobs
// ---------------------------------------------------------------------------
static Knobs g_knobs;
static thread_local int t_nbc = NBC_NONE;  // nonblocking initiation in progress (nbc_set)
static bool g_knobs_ok = false;
static uint64_t g_knobs_gen = 0;  // bumped by knobs_reload / topo_set: invalidates cached plans
static Topo g_topo{};

const Topo &topo() { return g_topo; }
void topo_set(const Topo &t) {
    g_topo = t;
    if (g_topo.nlevels < 0) g_topo.nlevels = 0;
    if (g_topo.nlevels > kTopoLevels) g_topo.nlevels = kTopoLevels;
    ++g_knobs_gen;
}

static bool env_set(const char *name, const char **v) {
    *v = getenv(name);
    return *v && **v;
}

// user_val_to_bytes (mv2_utils.c:27-70): a trailing K/M/G multiplies, as an int
static int64_t val_to_bytes(const char *v) {
    const size_t len = strlen(v);
    int64_t f = 1;
    const char last = v[len - 1];
    if (last == 'k' || last == 'K') f = 1 << 10;
    else if (last == 'm' || last == 'M') f = 1 << 20;
    else if (last == 'g' || last == 'G') f = 1 << 30;
    return (int64_t)(int)((int64_t)atoi(v) * f);
}

void knobs_reload() {
    Knobs k{};
    k.enable_shmem_collectives = 1;
    k.enable_shmem_allreduce = 1;
    k.enable_shmem_reduce = 1;
    k.enable_skip_search = 1;
    k.coll_skip_thr = 1024;
    k.allred_skip_small = 1;
    k.allred_skip_large = 1;
    k.enable_topo = 1;
    k.use_topo_allreduce = 1;
    k.topo_allred_min = 1;
    k.topo_allred_max = 2048;
    k.topo_allred_ppn = 1;
    k.use_topo_reduce = 0;
    k.topo_red_min = 1;
    k.topo_red_max = 2048;
    k.topo_red_ppn = 1;
    k.topo_red_nodes = 1;
    k.tree_degree = 4;
    k.allred_use_ring = 1;
    k.allred_ring_thr = (int64_t)2 << 20;
    k.allred_ring_ppn = 8;
    k.smp_use_cma = 1;
    k.use_knomial_reduce = 1;
    k.reduce_inter_k = -1;
    k.shmem_coll_max_msg = 32 * 1024;
    k.shmem_intra_reduce_msg = 1 << 11;
    k.red_scat_ring_thr = 131072;
    const char *v;
    int flag;
    // ch3_shmem_coll.c MV2_Read_env_vars, in its order where order matters
    if (env_set("MV2_USE_SHARED_MEM", &v) && atoi(v) <= 0) k.enable_shmem_collectives = 0;
    if (env_set("MV2_USE_SHMEM_ALLREDUCE", &v)) k.enable_shmem_allreduce = atoi(v);
    if (env_set("MV2_USE_SHMEM_REDUCE", &v)) k.enable_shmem_reduce = atoi(v);
    if (env_set("MV2_ENABLE_SKIP_TUNING_TABLE_SEARCH", &v)) k.enable_skip_search = !!atoi(v);
    if (env_set("MV2_COLL_SKIP_TABLE_THRESHOLD", &v)) {
        k.coll_skip_thr = atoi(v);  // a negative value keeps the threshold negative (:2328-2331)
    }
    if (env_set("MV2_ENABLE_ALLREDUCE_SKIP_LARGE_MESSAGE_TUNING_TABLE_SEARCH", &v)) k.allred_skip_large = !!atoi(v);
    if (env_set("MV2_ENABLE_ALLREDUCE_SKIP_SMALL_MESSAGE_TUNING_TABLE_SEARCH", &v)) k.allred_skip_small = !!atoi(v);
    if (env_set("MV2_USE_KNOMIAL_REDUCE", &v) && (flag = atoi(v)) >= 0) k.use_knomial_reduce = flag;
    if (env_set("MV2_USE_INTER_KNOMIAL_REDUCE_FACTOR", &v) && (flag = atoi(v)) >= 0) k.reduce_inter_k = flag;
    if (env_set("MV2_SHMEM_COLL_MAX_MSG_SIZE", &v) && (flag = atoi(v)) > 0) k.shmem_coll_max_msg = flag;
    if (env_set("MV2_INTRA_SHMEM_REDUCE_MSG", &v) && (flag = atoi(v)) >= 0) k.shmem_intra_reduce_msg = flag;
    if (env_set("MV2_ALLRED_USE_RING", &v)) k.allred_use_ring = atoi(v) > 0 ? 1 : 0;
    if (env_set("MV2_ALLREDUCE_RING_ALGO_PPN_THRESHOLD", &v) && (flag = atoi(v)) >= 1) k.allred_ring_ppn = flag;
    if (env_set("MV2_ALLREDUCE_RING_ALGO_THRESHOLD", &v)) {
        k.allred_ring_thr = val_to_bytes(v);
        if (k.allred_ring_thr < 0) k.allred_ring_thr = 0;
    }
    if (env_set("MV2_RED_SCAT_RING_ALGO_THRESHOLD", &v)) {
        k.red_scat_ring_thr = val_to_bytes(v);
        if (k.red_scat_ring_thr < 0) k.red_scat_ring_thr = 0;
    }
    if (env_set("MV2_SHMEM_REDUCE_TREE_DEGREE", &v)) k.tree_degree = atoi(v);
    // socket-aware collectives switch the topology-aware ones off (:3304-3320)
    if (env_set("MV2_ENABLE_SOCKET_AWARE_COLLECTIVES", &v) && atoi(v)) k.enable_topo = 0;
    if (env_set("MV2_ENABLE_TOPO_AWARE_COLLECTIVES", &v)) k.enable_topo = !!atoi(v);
    if (env_set("MV2_USE_TOPO_AWARE_ALLREDUCE", &v)) k.use_topo_allreduce = !!atoi(v);
    if (env_set("MV2_USE_TOPO_AWARE_REDUCE", &v)) k.use_topo_reduce = !!atoi(v);
    if (env_set("MV2_TOPO_AWARE_ALLREDUCE_MAX_MSG", &v)) k.topo_allred_max = atoi(v);
    if (env_set("MV2_TOPO_AWARE_ALLREDUCE_MIN_MSG", &v)) k.topo_allred_min = atoi(v);
    if (env_set("MV2_TOPO_AWARE_REDUCE_MAX_MSG", &v)) k.topo_red_max = atoi(v);
    if (env_set("MV2_TOPO_AWARE_REDUCE_MIN_MSG", &v)) k.topo_red_min = atoi(v);
    if (env_set("MV2_TOPO_AWARE_REDUCE_PPN_THRESHOLD", &v)) k.topo_red_ppn = atoi(v);
    if (env_set("MV2_TOPO_AWARE_REDUCE_NODE_THRESHOLD", &v)) k.topo_red_nodes = atoi(v);
    // CMA selects the reduce tables (reduce_tuning.c:1578-1629; ibv_param.c:716)
    if (env_set("MV2_SMP_USE_CMA", &v)) k.smp_use_cma = !!atoi(v);
    k.reduce_short_msg = 2048;
    k.redscat_comm_long = 524288;
    if (env_set("MPIR_CVAR_REDUCE_SHORT_MSG_SIZE", &v) || env_set("MPICH_REDUCE_SHORT_MSG_SIZE", &v))
        k.reduce_short_msg = atoi(v);
    if (env_set("MPIR_CVAR_REDSCAT_COMMUTATIVE_LONG_MSG_SIZE", &v) || env_set("MPICH_REDSCAT_COMMUTATIVE_LONG_MSG_SIZE", &v))
        k.redscat_comm_long = atoi(v);
    g_knobs = k;
    g_knobs_ok = true;
    ++g_knobs_gen;
}

const Knobs &knobs() {
    if (!g_knobs_ok) knobs_reload();
    return g_knobs;
}

const char *algo_name(int a) {
    static const char *names[ALG_COUNT] = {
        "none", "shmem_linear", "pt2pt_rs", "pt2pt_rd", "ring_wrapper", "topo_tree", "two_level_p2p",
        "binomial", "knomial", "redscat_gather", "rs_ring", "rs_rec_halving", "rs_pairwise", "rs_basic",
        "reduce_topo", "rs_noncomm_pof2", "rs_noncomm_rd"};
    return (a >= 0 && a < ALG_COUNT) ? names[a] : "?";
}

// ---------------------------------------------------------------------------
// symbolic expressions and their compilation to programs
// ---------------------------------------------------------------------------
namespace {

struct Sym {
    struct Node {
        int leaf;  // >= 0: rank operand
        int a, b;  // op(a = inout, b = in)
    };
    std::vector<Node> nodes;
    int leaf(int r) {
        nodes.push_back({r, -1, -1});
        return (int)nodes.size() - 1;
    }
    int op(int acc, int in) {
        nodes.push_back({-1, acc, in});
        return (int)nodes.size() - 1;
    }
    // returns the register holding e's value, or -1 on a malformed tree
    int emit(int e, Prog &p, unsigned &used) const {
        const Node &nd = nodes[e];
        if (nd.leaf >= 0) {
            if (used & (1u << nd.leaf)) return -1;
            used |= 1u << nd.leaf;
            return nd.leaf;
        }
        const int ra = emit(nd.a, p, used);
        const int rb = emit(nd.b, p, used);
        if (ra < 0 || rb < 0 || p.nsteps >= kMaxRanks - 1) return -1;
        p.dst[p.nsteps] = (uint8_t)ra;
        p.src[p.nsteps] = (uint8_t)rb;
        ++p.nsteps;
        return ra;
    }
    // Every program is compiled here, from one expression tree walked from its root: each step
    // belongs to res's tree and each register is one rank's operand, used once (emit refuses a
    // leaf twice).  device_util.h prog_eval's order-free shortcut folds exactly the registers a
    // program names, which equals the program's result only under that property, so it is checked
    // once more on the result: a tree with k leaves has k - 1 steps.
    bool compile(int e, Prog &p) const {
        memset(&p, 0, sizeof(p));
        unsigned used = 0;
        const int r = emit(e, p, used);
        if (r < 0) return false;
        p.res = (uint8_t)r;
        unsigned named = p.nsteps ? 0u : 1u << p.res;
        for (int k = 0; k < p.nsteps; ++k) named |= (1u << p.dst[k]) | (1u << p.src[k]);
        if (named != used || __builtin_popcount(used) != p.nsteps + 1) return false;
        return true;
    }
};

int pof2_of(int n) {
    int p = 1;
    while (p * 2 <= n) p *= 2;
    return p;
}

void single(ProgSet &ps, const Prog &p) {
    memset(&ps, 0, sizeof(ps));
    ps.nprog = 1;
    ps.blk = ~(uint64_t)0 >> 1;
    ps.p[0] = p;
}

bool single_expr(const Sym &s, int e, ProgSet &ps) {
    Prog p;
    if (!s.compile(e, p)) return false;
    single(ps, p);
    return true;
}

// LINEAR: ((x0 . x1) . x2) ... (reduce_shmem allreduce_osu.c:1569-1583,
// MPIR_Reduce_shmem_MV2 reduce_osu.c:1517-1532)
bool prog_linear(int n, ProgSet &ps) {
    Sym s;
    int acc = s.leaf(0);
    for (int i = 1; i < n; ++i) acc = s.op(acc, s.leaf(i));
    return single_expr(s, acc, ps);
}

// mv2_shm_tree_reduce (ch3_shmem_coll.c:4272-4359) over the members m[0..cnt) of one
// communicator (in its rank order), rooted at m[0]: every member with index % deg == 0 reduces
// members g+1 .. g+deg-1 in order; the root then reduces the group leaders deg, 2deg, ... in
// order.  val[r] = the expression rank r holds; the result lands in val[m[0]].
void shm_tree_sym(Sym &s, std::vector<int> &val, const int *m, int cnt, int deg) {
    for (int g = 0; g < cnt; g += deg)
        for (int i = g + 1; i < g + deg && i < cnt; ++i) val[m[g]] = s.op(val[m[g]], val[m[i]]);
    for (int g = deg; g < cnt; g += deg) val[m[0]] = s.op(val[m[0]], val[m[g]]);
}

// The topology-aware reduce to local rank 0 (allreduce_osu.c:2340-2361): one shm tree per
// level.  At level l the current communicator (all ranks at level 0, then the previous level's
// group leaders, in rank order) splits by each member's colour at l (0 past the levels); each
// group reduces into its first member, which leads it into level l+1; one group ends the walk
// (create_2level_comm.c:836-846: no leader communicator).
bool prog_tree(int n, int deg, ProgSet &ps) {
    if (deg < 1) deg = 1;
    const Topo &t = topo();
    Sym s;
    std::vector<int> val(n);
    for (int r = 0; r < n; ++r) val[r] = s.leaf(r);
    std::vector<int> cur(n);
    for (int r = 0; r < n; ++r) cur[r] = r;
    for (int lvl = 0;; ++lvl) {
        auto color = [&](int r) { return lvl < t.nlevels ? t.color[lvl][r] : 0; };
        std::vector<int> leaders;
        std::vector<bool> seen(cur.size(), false);
        for (size_t i = 0; i < cur.size(); ++i) {
            if (seen[i]) continue;
            int m[kMaxRanks], cnt = 0;
            for (size_t j = i; j < cur.size(); ++j)
                if (!seen[j] && color(cur[j]) == color(cur[i])) {
                    seen[j] = true;
                    m[cnt++] = cur[j];
                }
            shm_tree_sym(s, val, m, cnt, deg);
            leaders.push_back(cur[i]);
        }
        if (leaders.size() == 1) return single_expr(s, val[leaders[0]], ps);
        if (lvl > kTopoLevels) return false;
        cur = leaders;
    }
}

// MPIR_Reduce_binomial_MV2 (reduce_osu.c:577-643), commutative: relrank =
// (rank - root) mod n; at mask m a rank without bits below m receives from
// relrank | m and computes uop(tmp, recvbuf) (own value is inout)
// Non-commutative ops use lroot = 0 (the result is then sent to the root,
// :645-663) and uop(recvbuf, tmp): the received higher ranks are the inout.
bool prog_binomial(int n, int root, bool noncomm, ProgSet &ps) {
    if (noncomm) root = 0;
    Sym s;
    std::vector<int> cur(n);
    for (int r = 0; r < n; ++r) cur[r] = s.leaf((r + root) % n);
    for (int mask = 1; mask < n; mask <<= 1)
        for (int r = 0; r < n; ++r)
            if ((r & (2 * mask - 1)) == 0 && (r | mask) < n)
                cur[r] = noncomm ? s.op(cur[r | mask], cur[r]) : s.op(cur[r], cur[r | mask]);
    return single_expr(s, cur[0], ps);
}

// MPIR_Reduce_knomial_MV2 (reduce_osu.c:1639-1835) with the children of
// MPIR_Reduce_knomial_trace (:1569-1633).  Receives are posted in reverse
// src_array order and reduced in PMPI_Waitany completion order (:1747-1786);
// the order used here is the request-index order, which is what Waitany
// returns when the children's messages have all arrived.
int knomial_expr(Sym &s, int n, int root, int k, int r) {
    int mask = 1;
    while (mask < n) {
        if (r % (k * mask)) break;
        mask *= k;
    }
    mask /= k;
    std::vector<int> src;
    for (int m = mask; m > 0; m /= k)
        for (int j = 1; j < k; ++j)
            if (r + m * j < n) src.push_back(r + m * j);
    int acc = s.leaf((r + root) % n);
    for (int i = (int)src.size() - 1; i >= 0; --i) acc = s.op(acc, knomial_expr(s, n, root, k, src[i]));
    return acc;
}

bool prog_knomial(int n, int root, int k, ProgSet &ps) {
    Sym s;
    return single_expr(s, knomial_expr(s, n, root, k, 0), ps);
}

// Recursive-halving reduce-scatter over pof2 blocks as in
// MPIR_Allreduce_pt2pt_rs_MV2 (allreduce_osu.c:853-947) and
// MPIR_Reduce_redscat_gather_MV2 (reduce_osu.c:907-991): mask = 1, 2, ...;
// the lower newrank keeps the lower half of its index range; the received
// part is reduced as uop(tmp, recvbuf).  cur[nr][i] is newrank nr's partial
// of block i; returns the final owner's expression of each block.
void rs_halving(Sym &s, int pof2, std::vector<std::vector<int>> &cur, std::vector<int> &block_expr) {
    std::vector<int> send_idx(pof2, 0), recv_idx(pof2, 0), last_idx(pof2, pof2);
    std::vector<int> lo(pof2, 0), hi(pof2, pof2);
    for (int mask = 1; mask < pof2; mask <<= 1) {
        std::vector<std::vector<int>> prev = cur;
        for (int nr = 0; nr < pof2; ++nr) {
            const int nd = nr ^ mask;
            if (nr < nd) {
                send_idx[nr] = recv_idx[nr] + pof2 / (mask * 2);
                lo[nr] = recv_idx[nr];
                hi[nr] = send_idx[nr];
            } else {
                recv_idx[nr] = send_idx[nr] + pof2 / (mask * 2);
                lo[nr] = recv_idx[nr];
                hi[nr] = last_idx[nr];
            }
        }
        for (int nr = 0; nr < pof2; ++nr)
            for (int i = lo[nr]; i < hi[nr]; ++i) cur[nr][i] = s.op(prev[nr][i], prev[nr ^ mask][i]);
        for (int nr = 0; nr < pof2; ++nr) {
            send_idx[nr] = recv_idx[nr];
            if ((mask << 1) < pof2) last_idx[nr] = recv_idx[nr] + pof2 / (mask << 1);
        }
    }
    block_expr.assign(pof2, -1);
    for (int nr = 0; nr < pof2; ++nr) {
        // after the last step newrank nr holds exactly one block: [lo, hi)
        const int b = pof2 == 1 ? 0 : lo[nr];
        block_expr[b] = cur[nr][b];
    }
}

bool blocks_to_progset(const Sym &s, const std::vector<int> &blk_expr, size_t count, ProgSet &ps) {
    const int nb = (int)blk_expr.size();
    memset(&ps, 0, sizeof(ps));
    ps.nprog = nb;
    ps.blk = count / (size_t)nb;
    if (ps.blk == 0) ps.blk = 1;
    for (int b = 0; b < nb; ++b)
        if (blk_expr[b] < 0 || !s.compile(blk_expr[b], ps.p[b])) return false;
    return true;
}

// MPIR_Allreduce_pt2pt_rs_MV2 (allreduce_osu.c:633-1054) for builtin ops.
// Non-pof2 pre-step (:734-777): even r < 2rem sends to r+1, odd r computes
// uop(tmp = x_{r-1}, recv = x_r).  count < pof2 (:802): recursive doubling
// (every rank's own result); else recursive halving + doubling allgather.
// Non-commutative (user) ops always take recursive doubling; a step keeps the
// lower real rank on the left (:824-845: uop(recvbuf, tmp) when dst > rank).
bool prog_pt2pt_rs(int n, int me, size_t count, bool force_rd, ProgSet &ps, bool noncomm = false) {
    const int pof2 = pof2_of(n), rem = n - pof2;
    Sym s;
    std::vector<int> x(n);
    for (int r = 0; r < n; ++r) x[r] = s.leaf(r);
    std::vector<int> base(pof2);
    for (int nr = 0; nr < pof2; ++nr) base[nr] = nr < rem ? s.op(x[2 * nr + 1], x[2 * nr]) : x[nr + rem];
    if (force_rd || count < (size_t)pof2) {
        std::vector<int> cur = base;
        auto real = [&](int nr) { return nr < rem ? 2 * nr + 1 : nr + rem; };
        for (int mask = 1; mask < pof2; mask <<= 1) {
            std::vector<int> prev = cur;
            for (int nr = 0; nr < pof2; ++nr) {
                const int nd = nr ^ mask;
                cur[nr] = (!noncomm || real(nd) < real(nr)) ? s.op(prev[nr], prev[nd]) : s.op(prev[nd], prev[nr]);
            }
        }
        // post-step (:1003-1030): even r < 2rem takes the result of r+1
        const int r = (me < 2 * rem && me % 2 == 0) ? me + 1 : me;
        const int nr = r < 2 * rem ? r / 2 : r - rem;
        return single_expr(s, cur[nr], ps);
    }
    std::vector<std::vector<int>> cur(pof2, std::vector<int>(pof2));
    for (int nr = 0; nr < pof2; ++nr)
        for (int i = 0; i < pof2; ++i) cur[nr][i] = base[nr];
    std::vector<int> be;
    rs_halving(s, pof2, cur, be);
    return blocks_to_progset(s, be, count, ps);
}

// MPIR_Reduce_redscat_gather_MV2 (reduce_osu.c:718-1135): the pre-step runs
// the other way round (:849-894: odd r < 2rem sends to r-1, even r computes
// uop(tmp = x_{r+1}, recv = x_r)); the gather to the root only moves data.
bool prog_redscat_gather(int n, size_t count, ProgSet &ps) {
    const int pof2 = pof2_of(n), rem = n - pof2;
    Sym s;
    std::vector<int> x(n);
    for (int r = 0; r < n; ++r) x[r] = s.leaf(r);
    std::vector<std::vector<int>> cur(pof2, std::vector<int>(pof2));
    for (int nr = 0; nr < pof2; ++nr) {
        const int b = nr < rem ? s.op(x[2 * nr], x[2 * nr + 1]) : x[nr + rem];
        for (int i = 0; i < pof2; ++i) cur[nr][i] = b;
    }
    std::vector<int> be;
    rs_halving(s, pof2, cur, be);
    return blocks_to_progset(s, be, count, ps);
}

// MPIR_Allreduce_pt2pt_ring_MV2 (allreduce_osu.c:3925-3958): chunk c starts at
// rank c; hop k runs uop(in = own chunk of rank c+k, inout = received partial)
bool prog_ring_allreduce(int n, size_t count, ProgSet &ps) {
    Sym s;
    std::vector<int> be(n);
    for (int c = 0; c < n; ++c) {
        int acc = s.leaf(c);
        for (int k = 1; k < n; ++k) acc = s.op(acc, s.leaf((c + k) % n));
        be[c] = acc;
    }
    if (!blocks_to_progset(s, be, count, ps)) return false;
    ps.blk = count / (size_t)n;
    return true;
}

// MPIR_Reduce_scatter_ring(_2lvl) (red_scat_osu.c:1290-1336): block b starts at
// rank b+1; each later rank runs Reduce_local(in = received, inout = own chunk)
int rs_ring_expr(Sym &s, int n, int b) {
    int acc = s.leaf((b + 1) % n);
    for (int k = 2; k <= n; ++k) acc = s.op(s.leaf((b + k) % n), acc);
    return acc;
}

// MPIR_Reduce_scatter_Rec_Halving_MV2 (red_scat_osu.c:537-760): pre-step
// even r < 2rem sends to r+1, odd r: uop(tmp = x_{r-1}, results = x_r);
// new block i = old blocks of the ranks it stands for; halving from
// mask = pof2/2 down to 1, the lower newrank keeping the lower half.
int rs_rec_halving_expr(Sym &s, int n, int me) {
    const int pof2 = pof2_of(n), rem = n - pof2;
    std::vector<int> x(n);
    for (int r = 0; r < n; ++r) x[r] = s.leaf(r);
    std::vector<std::vector<int>> cur(pof2, std::vector<int>(pof2));
    for (int nr = 0; nr < pof2; ++nr) {
        const int b = nr < rem ? s.op(x[2 * nr + 1], x[2 * nr]) : x[nr + rem];
        for (int i = 0; i < pof2; ++i) cur[nr][i] = b;
    }
    std::vector<int> send_idx(pof2, 0), recv_idx(pof2, 0), last_idx(pof2, pof2), lo(pof2), hi(pof2);
    for (int mask = pof2 >> 1; mask > 0; mask >>= 1) {
        std::vector<std::vector<int>> prev = cur;
        for (int nr = 0; nr < pof2; ++nr) {
            const int nd = nr ^ mask;
            if (nr < nd) {
                send_idx[nr] = recv_idx[nr] + mask;
                lo[nr] = recv_idx[nr];
                hi[nr] = send_idx[nr];
            } else {
                recv_idx[nr] = send_idx[nr] + mask;
                lo[nr] = recv_idx[nr];
                hi[nr] = last_idx[nr];
            }
        }
        for (int nr = 0; nr < pof2; ++nr)
            for (int i = lo[nr]; i < hi[nr]; ++i) cur[nr][i] = s.op(prev[nr][i], prev[nr ^ mask][i]);
        for (int nr = 0; nr < pof2; ++nr) {
            send_idx[nr] = recv_idx[nr];
            last_idx[nr] = recv_idx[nr] + mask;
        }
    }
    const int nb = me < 2 * rem ? me / 2 : me - rem;  // new block holding my old block
    // the newrank whose final single-block range is nb
    for (int nr = 0; nr < pof2; ++nr)
        if ((pof2 == 1 ? 0 : lo[nr]) == nb) return cur[nr][nb];
    return -1;
}

// MPIR_Reduce_scatter_Pair_Wise_MV2 (red_scat_osu.c:867-989), commutative:
// own block, then uop(tmp = x_{me-i}, recvbuf) for i = 1 .. n-1
int rs_pairwise_expr(Sym &s, int n, int me) {
    int acc = s.leaf(me);
    for (int i = 1; i < n; ++i) acc = s.op(acc, s.leaf((me - i + n) % n));
    return acc;
}

// MPIR_Reduce_scatter_noncomm_MV2 (red_scat_osu.c:132-290), a power-of-two size with equal
// counts: the blocks are mirror-permuted (:90-103, :211-222), then at step k rank r and its peer
// r ^ 2^k split their current range of positions, the higher rank keeping the upper half, and
// both reduce the kept half as uop(in = the lower rank's partial, inout = the higher rank's)
// (:260-272).  Rank r ends at position mirror(r), i.e. with block r.
int rs_noncomm_pof2_expr(Sym &s, int n, int me) {
    std::vector<std::vector<int>> val(n, std::vector<int>(n));
    for (int r = 0; r < n; ++r)
        for (int p = 0; p < n; ++p) val[r][p] = s.leaf(r);
    std::vector<int> lo(n, 0), sz(n, n);
    for (int k = 0; (1 << k) < n; ++k) {
        std::vector<std::vector<int>> nv = val;
        for (int r = 0; r < n; ++r) {
            const int q = r ^ (1 << k), half = sz[r] / 2;
            const int keep = r > q ? lo[r] + half : lo[r];
            const int hi = std::max(r, q), low = std::min(r, q);
            for (int p = keep; p < keep + half; ++p) nv[r][p] = s.op(val[hi][p], val[low][p]);
            lo[r] = keep;
            sz[r] = half;
        }
        val.swap(nv);
    }
    return val[me][lo[me]];
}

// MPIR_Reduce_scatter_non_comm_MV2's recursive doubling (red_scat_osu.c:1478-1722), any size and
// counts: at mask 2^i every rank exchanges with rank ^ mask all blocks outside the partner's
// subtree [dst_tree_root, +mask); where the partner subtree is cut off by the size, the ranks of
// this subtree that got data hand their received blocks down to the others (:1592-1656); then
// uop(in = received, inout = results) when the partner subtree is the lower one, else
// uop(in = results, inout = received) (:1668-1720).  Expressions are per block; the result is
// block `me` on rank me.
int rs_noncomm_rd_expr(Sym &s, int n, int me) {
    std::vector<std::vector<int>> res(n, std::vector<int>(n)), rcv(n, std::vector<int>(n, -1));
    for (int r = 0; r < n; ++r)
        for (int b = 0; b < n; ++b) res[r][b] = s.leaf(r);
    for (int mask = 1, i = 0; mask < n; mask <<= 1, ++i) {
        std::vector<int> dtr(n), mtr(n);
        std::vector<bool> got(n, false);
        for (int r = 0; r < n; ++r) {
            dtr[r] = ((r ^ mask) >> i) << i;
            mtr[r] = (r >> i) << i;
        }
        auto outside = [&](int b, int root) { return b < root || b >= root + mask; };
        const std::vector<std::vector<int>> snap = res;
        for (int r = 0; r < n; ++r) {
            const int dst = r ^ mask;
            if (dst >= n) continue;
            for (int b = 0; b < n; ++b)
                if (outside(b, dtr[r])) rcv[r][b] = snap[dst][b];
            got[r] = true;
        }
        int k = 0;
        for (int j = mask; j; j >>= 1) ++k;
        --k;
        for (int tm = mask >> 1; tm; tm >>= 1, --k) {
            std::vector<std::pair<int, int>> moves;
            for (int r = 0; r < n; ++r) {
                if (dtr[r] + mask <= n) continue;
                const int npc = n - mtr[r] - mask, d = r ^ tm, root = (r >> k) << k;
                if (d > r && r < root + npc && d >= root + npc && d < n) moves.push_back({r, d});
            }
            for (const auto &mv : moves) {
                for (int b = 0; b < n; ++b)
                    if (outside(b, dtr[mv.second])) rcv[mv.second][b] = rcv[mv.first][b];
                got[mv.second] = true;
            }
        }
        for (int r = 0; r < n; ++r) {
            if (!got[r]) continue;
            for (int b = 0; b < n; ++b) {
                if (!outside(b, dtr[r]) || rcv[r][b] < 0) continue;
                res[r][b] = dtr[r] < mtr[r] ? s.op(res[r][b], rcv[r][b]) : s.op(rcv[r][b], res[r][b]);
            }
        }
    }
    return res[me][me];
}

// tuning-table index of a message size (allreduce_osu.c:3241-3277,
// reduce_osu.c:2556-2586): 0 below the smallest entry, the last entry above
// the largest, else log2 of the largest power of two <= nbytes over the smallest
int table_index(long nbytes, long minsz, int size_table) {
    const long maxsz = minsz << (size_table - 1);
    if (nbytes < minsz) return 0;
    if (nbytes > maxsz) return size_table - 1;
    int idx = 0;
    long v = nbytes / minsz;
    while (v > 1) {
        v >>= 1;
        ++idx;
    }
    return idx;
}

// FIND_PPN_INDEX (common_tuning.h:91-115) over the default tables' ppn
// configurations {1, 2, 16}: one node with n ranks -> 0 (n = 1), 1 (n = 2), 2 (n >= 3)
int ppn_conf(int n) { return n <= 1 ? 0 : (n == 2 ? 1 : 2); }

}  // namespace

// ---------------------------------------------------------------------------
// MPI_Reduce
// ---------------------------------------------------------------------------
enum { R_BINOM = 0, R_KNOM = 1, R_RSG = 2 };

// First entries (numproc <= n) of the default reduce tables
// (reduce_tuning.c:1563-1649, "Stampede" fall-back for an unlisted
// architecture): tuning/reduce/gen2{_cma}_INTEL_XEON_E5_2680_16_MLX_CX_FDR_{2,16}ppn.h
struct ReduceEntry {
    int minsz, size;        // smallest inter-leader message size, size_inter_table
    int k;                  // inter_k_degree
    int two_level[19];
    int inter[19];
};
static const ReduceEntry kRedCma2 = {
    4, 19, 4, {0, 1, 1, 1, 1, 1, 1, 1, 1, 1, 0, 0, 0, 1, 1, 1, 1, 1, 1},
    {R_RSG, R_BINOM, R_KNOM, R_KNOM, R_RSG, R_BINOM, R_BINOM, R_KNOM, R_KNOM, R_BINOM, R_BINOM, R_RSG, R_BINOM,
     R_RSG, R_KNOM, R_KNOM, R_BINOM, R_BINOM, R_BINOM}};
static const ReduceEntry kRedCma16 = {
    4, 19, 4, {1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 0, 0, 1, 1, 0, 0, 0, 0, 0},
    {R_KNOM, R_RSG, R_BINOM, R_RSG, R_RSG, R_BINOM, R_BINOM, R_KNOM, R_RSG, R_RSG, R_KNOM, R_RSG, R_BINOM, R_BINOM,
     R_KNOM, R_RSG, R_RSG, R_RSG, R_RSG}};
static const ReduceEntry kRed2 = {
    1, 18, 4, {1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 0, 0, 0, 0, 0, 0, 0, 0, 1},
    {R_RSG, R_KNOM, R_KNOM, R_BINOM, R_BINOM, R_BINOM, R_BINOM, R_KNOM, R_BINOM, R_RSG, R_BINOM, R_BINOM, R_BINOM,
     R_BINOM, R_BINOM, R_BINOM, R_BINOM, R_BINOM, R_RSG}};
static const ReduceEntry kRed16 = {
    1, 18, 4, {1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 0, 0, 0, 0, 0, 0, 1, 0, 0},
    {R_BINOM, R_KNOM, R_BINOM, R_BINOM, R_RSG, R_RSG, R_RSG, R_RSG, R_RSG, R_RSG, R_KNOM, R_KNOM, R_KNOM, R_KNOM,
     R_KNOM, R_KNOM, R_KNOM, R_BINOM, R_BINOM}};

static int reduce_k(const Knobs &K, const ReduceEntry *e) {
    int k = K.reduce_inter_k >= 0 ? K.reduce_inter_k : (e ? e->k : 4);
    return k < 2 ? 2 : k;  // factors 0 and 1 never terminate the reference's trace loop
}

static int reduce_fill(Plan *p, int algo, int n, int root, size_t count, int k, bool noncomm = false) {
    p->algo = algo;
    p->k = k;
    bool ok = false;
    switch (algo) {
    case ALG_SHMEM_LINEAR: ok = prog_linear(n, p->ps); break;
    case ALG_BINOMIAL: ok = prog_binomial(n, root, noncomm, p->ps); break;
    case ALG_KNOMIAL: ok = prog_knomial(n, root, k, p->ps); p->unpinned = n > 2; break;
    case ALG_REDSCAT_GATHER: ok = prog_redscat_gather(n, count, p->ps); break;
    case ALG_REDUCE_TOPO: ok = prog_tree(n, k, p->ps); break;
    default: break;
    }
    return ok ? 0 : E_INTERN;
}

// MPIR_Reduce_two_level_helper_MV2, one-node branch (reduce_osu.c:2082-2166)
static int reduce_helper(const Knobs &K, Plan *p, int n, int root, size_t count, int textent,
                         const ReduceEntry *e) {
    const long stride = (long)count * textent;
    const int k = reduce_k(K, e);
    p->via |= VIA_TWO_LEVEL_HELPER;
    if (stride <= K.shmem_intra_reduce_msg && K.enable_shmem_reduce) {
        // MPIR_Reduce_shmem_MV2 at local root 0 (then sent to the root), or the intra knomial
        // wrapper at 0 from the shmem slot size on (:2125-2133)
        if (stride < K.shmem_coll_max_msg) return reduce_fill(p, ALG_SHMEM_LINEAR, n, 0, count, k);
        return reduce_fill(p, ALG_KNOMIAL, n, 0, count, k);
    }
    return reduce_fill(p, K.use_knomial_reduce == 1 ? ALG_KNOMIAL : ALG_BINOMIAL, n, root, count, k);
}

static int plan_reduce_build(int n, int me, int root, size_t count, int tsize, int textent, Plan *p, int opk) {
    (void)me;
    memset(p, 0, sizeof(*p));
    if (n <= 1) return 0;
    const Knobs &K = knobs();
    const bool comm = opk != OPK_USER_NONCOMM, builtin = opk == OPK_BUILTIN;
    const long nbytes = (long)count * tsize;
    // topology-aware reduce (reduce_osu.c:2498-2506), off by default
    if (nbytes <= K.topo_red_max && nbytes >= K.topo_red_min && K.enable_skip_search && nbytes <= K.coll_skip_thr &&
        K.enable_topo && K.use_topo_reduce && comm && n >= K.topo_red_ppn && K.topo_red_nodes <= 1)
        return reduce_fill(p, ALG_REDUCE_TOPO, n, root, count, K.tree_degree < 1 ? 1 : K.tree_degree);
    // small messages: shmem + binomial two-level (:2508-2514); two-level needs a
    // commutative op, else binomial (:2628-2636)
    if (K.enable_shmem_reduce && K.enable_skip_search && nbytes <= K.coll_skip_thr)
        return comm ? reduce_helper(K, p, n, root, count, textent, nullptr)
                    : reduce_fill(p, ALG_BINOMIAL, n, root, count, 0, true);
    const ReduceEntry *e = ppn_conf(n) == 1 ? (K.smp_use_cma ? &kRedCma2 : &kRed2)
                                            : (K.smp_use_cma ? &kRedCma16 : &kRed16);
    const int idx = table_index(nbytes, e->minsz, e->size);
    const int k = reduce_k(K, e);
    if (e->two_level[idx])
        return comm ? reduce_helper(K, p, n, root, count, textent, e)
                    : reduce_fill(p, ALG_BINOMIAL, n, root, count, k, true);
    switch (e->inter[idx]) {
    case R_KNOM:  // commutative only (:2637-2644)
        return reduce_fill(p, comm ? ALG_KNOMIAL : ALG_BINOMIAL, n, root, count, k, !comm);
    case R_RSG:  // builtin op and count >= pof2 (:2645-2652)
        return reduce_fill(p, builtin && count >= (size_t)pof2_of(n) ? ALG_REDSCAT_GATHER : ALG_BINOMIAL, n, root,
                           count, k, !comm);
    default: return reduce_fill(p, ALG_BINOMIAL, n, root, count, k, !comm);
    }
}

// ---------------------------------------------------------------------------
// MPI_Allreduce
// ---------------------------------------------------------------------------
enum { A_RS = 0, A_RD = 1 };
enum { I_SHMEM = 0, I_P2P = 1 };
// First entries of the default allreduce tables (allreduce_tuning.c:1714-1762,
// tuning/allreduce/nemesis_INTEL_XEON_E5_2680_16_MLX_CX_FDR_{2,16}ppn.h): 18
// entries of 1 B .. 128 KiB for both the inter-leader and the intra-node lists
struct AllreduceEntry {
    int two_level[19];
    int inter[18];
    int intra[18];
};
static const AllreduceEntry kAr2 = {
    {1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 0, 0, 0, 0, 0, 0, 0},
    {A_RD, A_RD, A_RD, A_RS, A_RS, A_RS, A_RD, A_RD, A_RD, A_RD, A_RS, A_RS, A_RS, A_RS, A_RS, A_RS, A_RS, A_RS},
    {I_SHMEM, I_SHMEM, I_SHMEM, I_SHMEM, I_SHMEM, I_SHMEM, I_SHMEM, I_SHMEM, I_SHMEM, I_SHMEM, I_SHMEM, I_SHMEM,
     I_P2P, I_P2P, I_P2P, I_P2P, I_P2P, I_P2P}};
static const AllreduceEntry kAr16 = {
    {1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 0, 0, 0, 0, 0, 0, 0, 0, 0},
    {A_RS, A_RS, A_RS, A_RS, A_RS, A_RS, A_RS, A_RS, A_RS, A_RS, A_RS, A_RS, A_RS, A_RS, A_RS, A_RS, A_RS, A_RS},
    {I_SHMEM, I_SHMEM, I_SHMEM, I_SHMEM, I_SHMEM, I_SHMEM, I_SHMEM, I_SHMEM, I_P2P, I_P2P, I_P2P, I_P2P, I_P2P, I_P2P,
     I_P2P, I_P2P, I_P2P, I_P2P}};

// pt2pt_rs falls back to recursive doubling for user ops and count < pof2 (:802)
static int allreduce_fill(Plan *p, int algo, int n, int me, size_t count, int opk = OPK_BUILTIN) {
    if (algo == ALG_PT2PT_RS && (opk != OPK_BUILTIN || count < (size_t)pof2_of(n))) {
        algo = ALG_PT2PT_RD;
        p->via |= VIA_RS_ENTRY;
    }
    p->algo = algo;
    bool ok = false;
    switch (algo) {
    case ALG_SHMEM_LINEAR: ok = prog_linear(n, p->ps); break;
    case ALG_PT2PT_RS: ok = prog_pt2pt_rs(n, me, count, false, p->ps); break;
    case ALG_PT2PT_RD: ok = prog_pt2pt_rs(n, me, count, true, p->ps, opk == OPK_USER_NONCOMM); break;
    case ALG_RING: ok = count >= (size_t)n && prog_ring_allreduce(n, (count / n) * n, p->ps); break;
    default: break;
    }
    return ok ? 0 : E_INTERN;
}

// MPIR_Allreduce_reduce_shmem_MV2 (allreduce_osu.c:1486-1610): below the shmem slot the leader's
// linear reduction; from the slot size on (count x extent >= MV2_SHMEM_COLL_MAX_MSG_SIZE, :1521-1526)
// it calls MPICH's MPIR_Reduce_intra to local rank 0 on the node's shmem communicator (not node
// aware, so flat; reduce.c:865-894): redscat_gather for a builtin op above
// MPIR_CVAR_REDUCE_SHORT_MSG_SIZE with count >= pof2, else binomial (reduce.c:92-265 and :298-,
// which reduce in MVAPICH2's binomial / redscat_gather order).  The shmem broadcast then gives every
// rank local rank 0's result; the plan keeps algo = shmem (its counters) with the reduce in inner.
static int reduce_shmem_fill(Plan *p, int n, int me, size_t count, int tsize, int textent, int opk) {
    const Knobs &K = knobs();
    if ((long)count * textent < K.shmem_coll_max_msg) return allreduce_fill(p, ALG_SHMEM_LINEAR, n, me, count, opk);
    const long nbytes = (long)count * tsize;
    const bool rsg = nbytes > K.reduce_short_msg && opk == OPK_BUILTIN && count >= (size_t)pof2_of(n);
    const int rc = reduce_fill(p, rsg ? ALG_REDSCAT_GATHER : ALG_BINOMIAL, n, 0, count, 0, opk == OPK_USER_NONCOMM);
    p->inner = p->algo;
    p->algo = ALG_SHMEM_LINEAR;
    return rc;
}

static int plan_allreduce_build(int n, int me, size_t count, int tsize, int textent, bool in_place, int forced,
                                Plan *p, int opk) {
    memset(p, 0, sizeof(*p));
    if (n <= 1) return 0;
    const Knobs &K = knobs();
    if (forced == ALG_SHMEM_LINEAR) return reduce_shmem_fill(p, n, me, count, tsize, textent, opk);
    if (forced == ALG_PT2PT_RS || forced == ALG_PT2PT_RD || forced == ALG_RING)
        return allreduce_fill(p, forced, n, me, count, opk);
    // a non-commutative op fails every shortcut's is_commutative test and ends in
    // recursive doubling whatever the size (allreduce_osu.c:3359-3368, :3893-3898, :802)
    if (opk == OPK_USER_NONCOMM) return allreduce_fill(p, ALG_PT2PT_RD, n, me, count, opk);
    const long nbytes = (long)count * tsize;
    // ALLREDUCE_SKIP_SMALL_MESSAGE_TUNING_TABLES (allreduce_osu.c:118-160)
    bool tables = false;
    if (K.allred_skip_small) {
        if (nbytes <= K.topo_allred_max && nbytes >= K.topo_allred_min && K.enable_topo && K.use_topo_allreduce) {
            if (n < K.topo_allred_ppn) {
                tables = true;  // goto use_tables
            } else {
                p->algo = ALG_TOPO_TREE;
                p->k = K.tree_degree < 1 ? 1 : K.tree_degree;
                return prog_tree(n, p->k, p->ps) ? 0 : E_INTERN;
            }
        }
        if (!tables && K.enable_shmem_allreduce && K.enable_skip_search && nbytes <= K.coll_skip_thr)
            return reduce_shmem_fill(p, n, me, count, tsize, textent, opk);
    }
    // ALLREDUCE_SKIP_LARGE_MESSAGE_TUNING_TABLES (:163-188): the flat ring wrapper at low ppn
    if (!tables && K.allred_skip_large && K.allred_use_ring == 1 && K.allred_ring_thr <= nbytes &&
        n <= K.allred_ring_ppn) {
        p->algo = ALG_RING;
        if (count >= (size_t)n && !in_place) return prog_ring_allreduce(n, (count / n) * n, p->ps) ? 0 : E_INTERN;
        return 0;  // the wrapper runs pt2pt_rs (count < n, or MPI_IN_PLACE): see coll.cpp
    }
    // tuning tables (:3162-3373)
    const AllreduceEntry &e = ppn_conf(n) == 1 ? kAr2 : kAr16;
    const int idx = table_index(nbytes, 1, 18);
    if (e.two_level[idx]) {
        // MPIR_Allreduce_two_level_MV2 (:1687-1830) when shmem is usable, else recursive doubling
        if (!(K.enable_shmem_allreduce && K.enable_shmem_collectives))
            return allreduce_fill(p, ALG_PT2PT_RD, n, me, count, opk);
        const int iidx = table_index(nbytes, 1, 18);
        if (e.intra[iidx] == I_SHMEM) return reduce_shmem_fill(p, n, me, count, tsize, textent, opk);
        // reduce_p2p (:1616-1684): MPIR_Reduce_MV2 to local rank 0, then the shmem bcast
        Plan r;
        const int rc = plan_reduce_build(n, me, 0, count, tsize, textent, &r, opk);
        if (rc) return rc;
        *p = r;
        p->inner = r.algo;
        p->algo = ALG_TWO_LEVEL_P2P;
        return 0;
    }
    return allreduce_fill(p, e.inter[idx] == A_RD ? ALG_PT2PT_RD : ALG_PT2PT_RS, n, me, count, opk);
}

// Several nodes: the tuning-table step of MPIR_Allreduce_index_tuned_intra_MV2 (:3162-3290) for
// `ppn` ranks per node and `gsize` ranks in all, over every numproc entry of the default tables
// nemesis_INTEL_XEON_E5_2680_16_MLX_CX_FDR_{1,2,16}ppn.h (the 16-ppn one for ppn >= 3).
// comm_size_index (:3210-3228): the entry of floor_pof2(gsize), clamped to the table's first and
// last; the message-size index over 18 entries from 1 byte (:3240-3275).  Returns 0
// (is_two_level), ALG_PT2PT_RS / ALG_PT2PT_RD (flat over every rank).  The multicast helper falls
// back to recursive doubling (:3324-3338), keeping a two-level entry two-level.
namespace {
struct MnEntry {
    int numproc;
    const char *two_level;  // per size index: '1' = MPIR_Allreduce_two_level_MV2
    const char *inter;      // s = pt2pt_rs, d = pt2pt_rd, m = multicast helper (-> pt2pt_rd)
    const char *intra;      // h = reduce_shmem, p = reduce_p2p, s = pt2pt_rs, d = pt2pt_rd
};
// the tables' per-entry lists, one character per message-size index (1 B, 2 B, ... 128 KiB)
const MnEntry k1ppnTab[] = {
    {2, "000000000000000000", "dddddddddddddsdsss", "pppppppppppppppppp"},
    {4, "010000000000000000", "smdddddddddddsssss", "phpppppppppppppppp"},
    {8, "111111111110011000", "sddddddddddddsssss", "psshhhssshhpphhppp"},
    {16, "010101111101111000", "dsssddddmddddsssss", "ppppppdphpppphhppp"},
    {32, "000001001111111100", "dsdssddddddddsssss", "ppppppppshhshppppp"},
};
const MnEntry k2ppnTab[] = {
    {2, "111111111111000000", "dddsssddddssssssss", "hhhhhhhhhhhhpppppp"},
    {4, "111111111111100000", "dddddddddddddsssss", "hhhhhhhhhhhhhppppp"},
    {8, "111111111111000000", "sdddddddddddssssss", "hhhhhhshhhhhpppppp"},
    {16, "111111111101100000", "smdddddddddddsssss", "hhhdhhddhdphpppppp"},
    {32, "111111111111110000", "dddddddddddddsssss", "sdsshssshsshshpppp"},
};
const MnEntry k16ppnTab[] = {
    {16, "111111111100000000", "ssssssssssssssssss", "hhhhhhhhpppppppppp"},
    {32, "111111111111000000", "sdddddddmdddssssss", "hhhhhhhhhpdppppppp"},
    {64, "111111111111100000", "dddmdddmmddddsssss", "hhhhhhhhhssssppppp"},
    {128, "111111111111100000", "sddddddddddddsssss", "hhshhshhspdsdppppp"},
    {256, "111111111111110000", "dmdsddmddmdmdsssss", "dhhpsshhshshsspppp"},
    {512, "111111111111111000", "dmsdddmmmddddsssss", "shhphphhhsdssppppp"},
    {1024, "111111111111110000", "dsmdsmddmdmddsssss", "phhphhhshshspppppp"},
};
}  // namespace

int mn_allreduce_table(int ppn, int gsize, long nbytes, int *intra, int *inter) {
    const int conf = ppn_conf(ppn);
    const MnEntry *tab = conf == 0 ? k1ppnTab : conf == 1 ? k2ppnTab : k16ppnTab;
    const int ntab = conf == 2 ? (int)(sizeof(k16ppnTab) / sizeof(k16ppnTab[0])) : 5;
    int ci = 0;  // comm_size_index
    if (gsize > tab[ntab - 1].numproc) {
        ci = ntab - 1;
    } else {
        for (int v = pof2_of(gsize); v > tab[0].numproc; v >>= 1) ++ci;
    }
    const MnEntry &e = tab[ci];
    const int idx = table_index(nbytes, 1, 18);
    const int a = e.inter[idx] == 's' ? ALG_PT2PT_RS : ALG_PT2PT_RD;
    // one rank per node: the two-level algorithm is its leaders' algorithm over every rank
    // (MPIR_Allreduce_two_level_MV2 :1750-1780 with nothing to reduce or broadcast in a node)
    if (e.two_level[idx] != '1' || ppn <= 1) return a;
    int in = MN_INTRA_SHMEM;
    switch (e.intra[idx]) {
    case 'p': in = MN_INTRA_P2P; break;
    case 's': in = MN_INTRA_RS; break;
    case 'd': in = MN_INTRA_RD; break;
    default: break;
    }
    // 16 ppn, numproc 16 entry: the node's one-node plan for its ppn ranks reads this same entry
    // (same intra function, plus its own checks), so the node step is that plan
    if (conf == 2 && ci == 0) in = MN_INTRA_NODE;
    if (intra) *intra = in;
    if (inter) *inter = a;
    return 0;
}

// Several nodes: MPIR_Reduce_index_tuned_intra_MV2's table step (reduce_osu.c:2516-2620) over the
// tables MVAPICH2 falls back to for an unlisted architecture (reduce_tuning.c:1563-1649, the
// "Stampede" branch): tuning/reduce/gen2{_cma}_INTEL_XEON_E5_2680_16_MLX_CX_FDR_{1,2,16}ppn.h, the
// first 5 / 6 / 6 numproc entries, as tests/golden/gen_mn_reduce_tables.py reads them.  Per entry:
// numproc, inter_k_degree, intra_k_degree, is_two_level_reduce per inter size index, the
// inter-leader list (smallest size, function per index: b binomial, k inter-knomial wrapper,
// r redscat_gather) and the intra-node list (h MPIR_Reduce_shmem_MV2, b binomial, i intra-knomial
// wrapper).  The lists hold size_inter_table / size_intra_table entries (the headers carry one more).
namespace {
struct MnRedEntry {
    int numproc, k, intra_k;
    const char *two_level;
    int inter_min;
    const char *inter;
    int intra_min;
    const char *intra;
};
const MnRedEntry kMnRedCma1[] = {
    {2, 4, 4, "111111111111111010", 1, "bbrkkbkkbbbkbrbbbb", 1, "bhbhbhhihiibiiihih"},
    {4, 4, 4, "111111111111010000", 1, "kkkbrbrkbrkbkrbbbb", 1, "bhihbiibhibhhihhhh"},
    {8, 4, 4, "111111111111011111", 1, "brrrrrrkbbkkkrkbbr", 1, "bbbbbbbbiihbhbbbib"},
    {16, 4, 4, "111111111111000111", 1, "bkkkkbkkkrbkkkbbbb", 1, "ibbhbbbbbbbihhhbhi"},
    {32, 4, 4, "111111111111000101", 1, "kkrbkrbrbbrrkbbbbr", 1, "bbhbibbiiihbhhhhhi"},
};
const MnRedEntry kMnRedCma2[] = {
    {2, 4, 4, "0111111111000111111", 4, "rbkkrbbkkbbrbrkkbbb", 4, "hhhiibihhhhhhbhbhh"},
    {2, 4, 4, "111111111100110111", 1, "rbbkbrkrbkbrrrkrrr", 1, "hihhbhbhhihhhhhhhh"},
    {4, 4, 4, "111111111111111100", 1, "rrbbrbbkbrbkkrkbbb", 1, "bihihihhihiihhhhhh"},
    {8, 4, 4, "111111111111111111", 1, "bkbbbrbbbbkkkrbbbb", 1, "biihibihhibhhhhhbb"},
    {16, 4, 4, "111111111111111111", 1, "brrrrrkkkrkkkkbbbb", 1, "ihihhhibihbhhhhhbb"},
    {32, 4, 4, "111111111111111101", 1, "rkkkkbkkkrrkkrbbbb", 1, "iiiibhiibihhhhhhhb"},
};
const MnRedEntry kMnRedCma16[] = {
    {16, 4, 4, "1111111111001100000", 4, "krbrrbbkrrkrbbkrrrr", 4, "ihhbbhbhihhhiiihhh"},
    {16, 4, 4, "111111111100000000", 1, "bkkbkkbrkkkbbbbbrr", 1, "ihbhhhhbibhhhhhhhh"},
    {32, 4, 4, "111111111111111111", 1, "kbkrrrkbkrkrkrkkkb", 1, "bhihbbhihbbbhhhhhb"},
    {64, 4, 4, "111111111111111111", 1, "rbbkrrrrkkbkkkbbbb", 1, "bihbbbiihbhhhhhhhb"},
    {128, 4, 4, "111111111111111111", 1, "rkbbbkkbbbrbkkkbbb", 1, "bbihhihibbiihhhhhb"},
    {256, 4, 4, "111111111111111100", 1, "brbrkkkkbkrbkkbbbb", 1, "hihiiihhbhbihhhhhh"},
};
const MnRedEntry kMnRed1[] = {
    {2, 4, 4, "111111111111110000", 1, "kkkbrkbbkkrrbrbbbk", 1, "iiiiiibhbhbihihhhh"},
    {4, 4, 4, "111111111111010010", 1, "kkrkbkrbbkrkkrbbbb", 1, "iihiihihiiihhbhhbh"},
    {8, 4, 4, "111111111111111110", 1, "bkrbbbbkkbkkkrkbbb", 1, "hihhhhhbhhbbbibbbh"},
    {16, 4, 4, "111111111111000011", 1, "kkkkbkkkkkrkkkbbbb", 1, "hhhhihhhhbbbhhhhbi"},
    {32, 4, 4, "111111111111000001", 1, "krrbkrbkkkrkkbbbbr", 1, "ihbbbhhbbbbbhhhhhb"},
};
const MnRedEntry kMnRed2[] = {
    {2, 4, 4, "111111111100000000", 1, "rkkbbbbkbrbbbbbbbb", 1, "bihihbhhhhhhhhhhhh"},
    {4, 4, 4, "111111111111111100", 1, "kbrrrrrkrbrrbrbbbb", 1, "bhiihbibhiiihhhhhh"},
    {8, 4, 4, "111111111111111100", 1, "brrrbrkkkbbrkrbbbb", 1, "iihiibhhihhihhhhhh"},
    {16, 4, 4, "111111111111011100", 1, "rrkrkrrkkkkkkrbkbb", 1, "iibihiiiibhhhhhhhh"},
    {32, 4, 4, "111111111111111100", 1, "rrrkkkrrrbbrkbbbbb", 1, "ibbbiibiibihhhhhhh"},
    {64, 4, 4, "111111111111011100", 1, "kbkkkkkbbrrkkkbbbb", 1, "bihibbiihhibhhhhhh"},
};
const MnRedEntry kMnRed16[] = {
    {16, 4, 4, "111111111100000010", 1, "bkbbrrrrrrkkkkkkkb", 1, "hiihbiihhihhhhhhhh"},
    {32, 4, 4, "111111111111011000", 1, "kkrbrrrkbkrkkbbkkb", 1, "bhbiibiihhbhhhihhh"},
    {64, 4, 4, "111111111111010010", 1, "kbkrrkkkbkbbkkkkbb", 1, "iihihhbbhhhhhhhhih"},
    {128, 4, 4, "111111111111010110", 1, "kkrrkrrkkkkkkkkbbb", 1, "hibihbbihiihhhhiih"},
    {256, 4, 4, "111111111111010110", 1, "kkkrbkkkkbbkkkkbrb", 1, "bihbhibhbbbhhhhiih"},
    {512, 4, 4, "111111111111111111", 1, "kbrkkkkrkbkbkkbbbb", 1, "iihhhhhhhhibihiiib"},
};
}  // namespace

int mn_reduce_table(int ppn, int gsize, long nbytes, MnReduceCell *c) {
    const Knobs &K = knobs();
    // FIND_PPN_INDEX over {1, 2, 16} (reduce_osu.c:2517, common_tuning.h:91-115)
    const int conf = ppn_conf(ppn);
    const MnRedEntry *tab = conf == 0 ? (K.smp_use_cma ? kMnRedCma1 : kMnRed1)
                          : conf == 1 ? (K.smp_use_cma ? kMnRedCma2 : kMnRed2)
                                      : (K.smp_use_cma ? kMnRedCma16 : kMnRed16);
    const int ntab = conf == 0 ? 5 : 6;
    // comm_size_index (:2528-2546): clamped to the table's ends, else log2 of floor_pof2(size) over
    // floor_pof2(the first entry's numproc) — an index, not a numproc match (the CMA 2- and 16-ppn
    // tables list their first numproc twice, so e.g. 32 ranks at 16 ppn read the second "16" entry)
    int ci;
    if (gsize < tab[0].numproc) {
        ci = 0;
    } else if (gsize > tab[ntab - 1].numproc) {
        ci = ntab - 1;
    } else {
        const int lmin = pof2_of(tab[0].numproc), l = pof2_of(gsize);
        ci = 0;
        for (int v = l; v > lmin; v >>= 1) ++ci;
        if (l < lmin) ci = 0;
    }
    const MnRedEntry &e = tab[ci];
    const int ni = (int)strlen(e.inter), nj = (int)strlen(e.intra);
    const int ii = table_index(nbytes, e.inter_min, ni), ij = table_index(nbytes, e.intra_min, nj);
    c->entry = ci;
    c->two_level = e.two_level[ii] == '1';
    c->inter = e.inter[ii] == 'k' ? ALG_KNOMIAL : e.inter[ii] == 'r' ? ALG_REDSCAT_GATHER : ALG_BINOMIAL;
    c->intra = e.intra[ij] == 'h' ? ALG_SHMEM_LINEAR : e.intra[ij] == 'i' ? ALG_KNOMIAL : ALG_BINOMIAL;
    // mv2_reduce_inter_knomial_factor (:2600-2607): MV2_USE_INTER_KNOMIAL_REDUCE_FACTOR, else the
    // entry's inter_k_degree; both knomial wrappers use it (:1841-1890)
    const int k = K.reduce_inter_k >= 0 ? K.reduce_inter_k : e.k;
    c->k = k < 2 ? 2 : k;  // factors 0 and 1 never terminate the reference's trace loop
    return 0;
}

int plan_reduce_forced(int n, int root, size_t count, int algo, int k, Plan *p, bool noncomm) {
    memset(p, 0, sizeof(*p));
    if (n <= 1) return 0;
    return reduce_fill(p, algo, n, root, count, k < 2 ? 2 : k, noncomm);
}

// ---------------------------------------------------------------------------
// MPI_Reduce_scatter (commutative ops; red_scat_osu.c:1859-1896)
// ---------------------------------------------------------------------------
// MPIR_Reduce_scatter_MV2's choice for a commutative op over n ranks (red_scat_osu.c:1859-1893): the
// ring from MV2_RED_SCAT_RING_ALGO_THRESHOLD (for node-major ranks the cyclic-hostfile test never
// holds), else the default table (red_scat_tuning.c:214-287), its entry the first numproc >= n (the
// last beyond), the function the first whose max >= nbytes among the entry's declared
// size_inter_table rows (:1877-1884: numproc 128 / 256 / 512 list a ring row but declare two rows,
// so recursive halving runs up to the ring threshold there).  MPIR_Reduce_scatter_ring_2lvl runs
// the plain ring's order for the identity rank list (:1190-1300 against :1026-1180).
int reduce_scatter_table(int n, long nbytes) {
    if (knobs().red_scat_ring_thr <= nbytes) return ALG_RS_RING;
    constexpr long kAll = 0x7fffffffffffffffL;
    static const struct {
        int numproc;
        long basic, halving, pairwise;  // inclusive upper bounds; the ring beyond
    } tab[] = {{8, 256, 16384, 65536},   {16, 64, 65536, 65536},   {32, 64, 131072, 131072},
               {64, 1024, 262144, 262144}, {128, 128, kAll, kAll}, {256, 128, kAll, kAll},
               {512, 256, kAll, kAll}};
    const int last = (int)(sizeof(tab) / sizeof(tab[0])) - 1;
    int r = 0;
    while (r < last && n > tab[r].numproc) ++r;
    if (nbytes <= tab[r].basic) return ALG_RS_BASIC;
    if (nbytes <= tab[r].halving) return ALG_RS_REC_HALVING;
    if (nbytes <= tab[r].pairwise) return ALG_RS_PAIRWISE;
    return ALG_RS_RING;
}

int reduce_scatter_algo(int n, long nbytes) {
    if (t_nbc == NBC_IREDUCE_SCATTER) return ALG_RS_PAIRWISE;
    if (t_nbc == NBC_IREDUCE_SCATTER_BLOCK)
        return nbytes < knobs().redscat_comm_long ? ALG_RS_REC_HALVING : ALG_RS_PAIRWISE;
    return reduce_scatter_table(n, nbytes);
}

// A non-commutative op's reduce-scatter: the power-of-two / equal-count special case (the mirror-
// permuted recursive halving) or recursive doubling.  The blocking MPIR_Reduce_scatter_non_comm_MV2
// (red_scat_osu.c:1367-1760), MPI_Ireduce_scatter's MPIR_Ireduce_scatter_tune_helper_MV2
// (ired_scat_osu.c:191-209: MPIR_Ireduce_scatter_noncomm :29-151 / MPIR_Ireduce_scatter_rec_dbl,
// ired_scat.c:496-752), MPIR_Reduce_scatter_block_intra (red_scat_block.c:614-640) and
// MPIR_Ireduce_scatter_block_intra (ired_scat_block.c:910-920; block counts are always equal) all
// make this choice, and their schedules reduce in the same order (op(received, mine) on the
// higher rank, op(mine, received) on the lower; the rec_dbl non-power-of-two hand-off inside subtrees)
static int plan_rs_noncomm(int n, int me, const size_t *counts, Plan *p) {
    int pof2 = 1;
    while (pof2 < n) pof2 <<= 1;
    bool regular = true;
    for (int j = 0; j + 1 < n; ++j) regular = regular && counts[j] == counts[j + 1];
    Sym s;
    int e;
    if (pof2 == n && regular) {
        p->algo = ALG_RS_NONCOMM_POF2;
        e = rs_noncomm_pof2_expr(s, n, me);
    } else {
        p->algo = ALG_RS_NONCOMM_RD;
        e = rs_noncomm_rd_expr(s, n, me);
    }
    return single_expr(s, e, p->ps) ? 0 : E_INTERN;
}

static int plan_reduce_scatter_build(int n, int me, const size_t *counts, int tsize, int textent, Plan *p,
                                     int opk) {
    memset(p, 0, sizeof(*p));
    if (n <= 1) return 0;
    size_t total = 0;
    for (int j = 0; j < n; ++j) total += counts[j];
    // MPIR_Reduce_scatter_MV2 sends every non-commutative op to MPIR_Reduce_scatter_non_comm_MV2
    // (red_scat_osu.c:1895-1898)
    if (opk == OPK_USER_NONCOMM) return plan_rs_noncomm(n, me, counts, p);
    const int algo = reduce_scatter_table(n, (long)total * tsize);
    p->algo = algo;
    Sym s;
    switch (algo) {
    case ALG_RS_RING: return single_expr(s, rs_ring_expr(s, n, me), p->ps) ? 0 : E_INTERN;
    case ALG_RS_PAIRWISE: return single_expr(s, rs_pairwise_expr(s, n, me), p->ps) ? 0 : E_INTERN;
    case ALG_RS_REC_HALVING: {
        const int e = rs_rec_halving_expr(s, n, me);
        return (e >= 0 && single_expr(s, e, p->ps)) ? 0 : E_INTERN;
    }
    default: {
        // MPIR_Reduce_MV2(total, root 0) then a scatter (:326-413)
        Plan r;
        const int rc = plan_reduce_build(n, 0, 0, total, tsize, textent, &r, opk);
        if (rc) return rc;
        p->ps = r.ps;
        p->inner = r.algo;
        p->k = r.k;
        p->unpinned = r.unpinned;
        p->via = r.via;
        return 0;
    }
    }
}

// ---------------------------------------------------------------------------
// Nonblocking collectives (one node, <= 8 ranks: the first row of each default
// nonblocking table, i.e. the unlisted-architecture "RI" tables)
// ---------------------------------------------------------------------------
void nbc_set(int kind) { t_nbc = kind; }
int nbc_kind() { return t_nbc; }

// MPIR_Iallreduce_intra_MV2 (iallreduce_osu.c:186-261) -> iallreduce_tuning.c:184-190:
// MPIR_Iallreduce_naive (iallreduce.c:109-139) = MPIR_Ireduce_intra to rank 0
// (ireduce.c:700-731: redscat_gather for builtin ops above
// MPIR_CVAR_REDUCE_SHORT_MSG_SIZE with count >= pof2, else binomial) + MPIR_Ibcast:
// every rank ends with rank 0's result.  The schedules reduce like the blocking
// algorithms (ireduce.c:219-224 binomial; :408-439, :524 redscat_gather).
static int plan_iallreduce_build(int n, int me, size_t count, int tsize, Plan *p, int opk) {
    (void)me;
    memset(p, 0, sizeof(*p));
    if (n <= 1) return 0;
    const long nbytes = (long)count * tsize;
    if (nbytes > knobs().reduce_short_msg && opk == OPK_BUILTIN && count >= (size_t)pof2_of(n))
        return reduce_fill(p, ALG_REDSCAT_GATHER, n, 0, count, 0);
    return reduce_fill(p, ALG_BINOMIAL, n, 0, count, 0, opk == OPK_USER_NONCOMM);
}

// MPIR_Ireduce_intra_MV2 (ireduce_osu.c:115-) -> ireduce_tuning.c default first row:
// MPIR_Ireduce_binomial (its tune helper only diverts redscat_gather, ireduce_osu.c:97-105)
static int plan_ireduce_build(int n, int root, size_t count, Plan *p, int opk) {
    memset(p, 0, sizeof(*p));
    if (n <= 1) return 0;
    return reduce_fill(p, ALG_BINOMIAL, n, root, count, 0, opk == OPK_USER_NONCOMM);
}

// MPI_Ireduce_scatter: MPIR_Ireduce_scatter_MV2 -> ired_scat_tuning.c default first row:
// MPIR_Ireduce_scatter_pairwise for commutative ops (ired_scat_osu.c:187-190; the
// schedule reduces like the blocking Pair_Wise, ired_scat.c:404-440).
// MPI_Ireduce_scatter_block: MPICH's MPIR_Ireduce_scatter_block_intra
// (ired_scat_block.c:882-920): recursive halving below
// MPIR_CVAR_REDSCAT_COMMUTATIVE_LONG_MSG_SIZE, pairwise from it (the schedules
// reduce like the blocking Rec_Halving / Pair_Wise, ired_scat_block.c:150-215).
static int plan_ireduce_scatter_build(int n, int me, const size_t *counts, int tsize, bool block, Plan *p, int opk) {
    memset(p, 0, sizeof(*p));
    if (n <= 1) return 0;
    if (opk == OPK_USER_NONCOMM) return plan_rs_noncomm(n, me, counts, p);
    size_t total = 0;
    for (int j = 0; j < n; ++j) total += counts[j];
    const long nbytes = (long)total * tsize;
    p->algo = (block && nbytes < knobs().redscat_comm_long) ? ALG_RS_REC_HALVING : ALG_RS_PAIRWISE;
    Sym s;
    if (p->algo == ALG_RS_PAIRWISE) return single_expr(s, rs_pairwise_expr(s, n, me), p->ps) ? 0 : E_INTERN;
    const int e = rs_rec_halving_expr(s, n, me);
    return (e >= 0 && single_expr(s, e, p->ps)) ? 0 : E_INTERN;
}

// ---------------------------------------------------------------------------
// plan cache: a plan is a pure function of its arguments and the knobs, and
// latency-bound loops repeat the same call, so the last plans of this thread
// are kept (the symbolic run costs 3-6 us per call on the host).
// ---------------------------------------------------------------------------
namespace {
struct PlanKey {
    int32_t coll, n, me, root, tsize, textent, in_place, forced, opk, pad;
    uint64_t count, gen;
    uint64_t counts[kMaxRanks];
};
constexpr int kPlanCache = 16;
struct PlanCache {
    PlanKey key[kPlanCache];
    Plan plan[kPlanCache];
    int used = 0, next = 0;
};
thread_local PlanCache t_cache;

PlanKey make_key(int coll, int n, int me, int root, size_t count, const size_t *counts, int tsize, int textent,
                 bool in_place, int forced, int opk) {
    PlanKey k;
    memset(&k, 0, sizeof(k));  // padding included: keys are compared bytewise
    k.coll = coll;
    k.n = n;
    k.me = me;
    k.root = root;
    k.tsize = tsize;
    k.textent = textent;
    k.in_place = in_place;
    k.forced = forced;
    k.opk = opk;
    k.count = count;
    knobs();
    k.gen = g_knobs_gen;
    if (counts)
        for (int j = 0; j < n && j < kMaxRanks; ++j) k.counts[j] = counts[j];
    return k;
}

template <class F>
int cached(const PlanKey &k, Plan *p, F build) {
    PlanCache &c = t_cache;
    for (int i = 0; i < c.used; ++i)
        if (!memcmp(&c.key[i], &k, sizeof(k))) {
            *p = c.plan[i];
            return 0;
        }
    const int rc = build();
    if (rc) return rc;
    const int i = c.next;
    c.key[i] = k;
    c.plan[i] = *p;
    c.next = (c.next + 1) % kPlanCache;
    if (c.used < kPlanCache) ++c.used;
    return 0;
}
}  // namespace

int plan_allreduce(int n, int me, size_t count, int tsize, int textent, bool in_place, int forced, Plan *p, int opk) {
    if (t_nbc == NBC_IALLREDUCE && !forced)
        return cached(make_key(3, n, me, 0, count, nullptr, tsize, textent, in_place, 0, opk), p,
                      [&] { return plan_iallreduce_build(n, me, count, tsize, p, opk); });
    return cached(make_key(0, n, me, 0, count, nullptr, tsize, textent, in_place, forced, opk), p,
                  [&] { return plan_allreduce_build(n, me, count, tsize, textent, in_place, forced, p, opk); });
}

int plan_reduce(int n, int me, int root, size_t count, int tsize, int textent, Plan *p, int opk) {
    if (t_nbc == NBC_IREDUCE)
        return cached(make_key(4, n, me, root, count, nullptr, tsize, textent, false, 0, opk), p,
                      [&] { return plan_ireduce_build(n, root, count, p, opk); });
    return cached(make_key(1, n, me, root, count, nullptr, tsize, textent, false, 0, opk), p,
                  [&] { return plan_reduce_build(n, me, root, count, tsize, textent, p, opk); });
}

int rs_noncomm_expr(int n, int me, bool pof2_equal, std::vector<ExprNode> &nodes) {
    Sym s;
    const int e = pof2_equal ? rs_noncomm_pof2_expr(s, n, me) : rs_noncomm_rd_expr(s, n, me);
    nodes.clear();
    nodes.reserve(s.nodes.size());
    for (const Sym::Node &nd : s.nodes) nodes.push_back(ExprNode{nd.leaf, nd.a, nd.b});
    return e;
}

int plan_binomial(int n, int root, Plan *p, bool noncomm) {
    memset(p, 0, sizeof(*p));
    if (n <= 1) return 0;
    return reduce_fill(p, ALG_BINOMIAL, n, root, 0, 0, noncomm);
}

int plan_reduce_scatter(int n, int me, const size_t *counts, int tsize, int textent, Plan *p, int opk) {
    if (n > kMaxRanks) return plan_reduce_scatter_build(n, me, counts, tsize, textent, p, opk);
    if (t_nbc == NBC_IREDUCE_SCATTER || t_nbc == NBC_IREDUCE_SCATTER_BLOCK) {
        const bool block = t_nbc == NBC_IREDUCE_SCATTER_BLOCK;
        return cached(make_key(block ? 6 : 5, n, me, 0, 0, counts, tsize, textent, false, 0, opk), p,
                      [&] { return plan_ireduce_scatter_build(n, me, counts, tsize, block, p, opk); });
    }
    return cached(make_key(2, n, me, 0, 0, counts, tsize, textent, false, 0, opk), p,
                  [&] { return plan_reduce_scatter_build(n, me, counts, tsize, textent, p, opk); });
}

}  // namespace mv2
