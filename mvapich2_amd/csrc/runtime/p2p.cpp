// p2p.cpp — point-to-point messages on device (or host) buffers between the
// ranks of one node: MPI_Send / MPI_Recv / MPI_Isend / MPI_Irecv.
//
// Reference: the ch3 device-buffer pt2pt path (MPIDI_CH3_EagerContigSend,
// ch3u_eager.c:153, with CUDA IPC eager/rendezvous in ibv_cuda_ipc.c and the
// matching queues of ch3u_recvq.c: posted + unexpected, non-overtaking
// per (source, tag, comm)).
//
// Here:
//   * one FIFO channel per ordered pair (src -> dst): kP2PSlots chunk records
//     in the /dev/shm control segment (world.h P2PChan) and kP2PSlots data
//     slots of kP2PChunk bytes in dst's uncached, IPC-exported P2P arena;
//   * the sender copies a chunk straight into the destination GPU's slot
//     (hipMemcpyAsync over xGMI into the peer mapping), waits for the copy,
//     then publishes the record (release) — a send completes once its last
//     chunk is in the receiver's arena (eager through the ring; messages
//     larger than the ring flow as the receiver frees slots);
//   * the receiver matches a message when its first chunk arrives against the
//     posted receives in posting order (MPI_ANY_SOURCE / MPI_ANY_TAG), else
//     drains it into an unexpected-message buffer so later messages keep
//     flowing; a receive posted later takes the earliest matching unexpected
//     message (arrival order), so per-(source, tag) order is preserved;
//   * progress is made inside Wait/Test of any request (and blocking calls).
// Copies run on their own stream so a pending nonblocking collective never
// blocks point-to-point progress.
//
// Ranks are global.  Between nodes (the reference's netmod path) a message
// travels on the rank mesh (internode.cpp mesh_setup: one TCP stream per pair of ranks on
// different nodes): a 24-byte header {source, tag, bytes}, then the payload, staged through host
// memory on both sides; the receiver matches the header against the same posted / unexpected
// queues, so MPI_ANY_SOURCE and per-(source, tag) order hold across both transports.
#include <hip/hip_runtime.h>
#include <sched.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <chrono>
#include <deque>
#include <list>
#include <unordered_map>
#include <vector>

#include <errno.h>
#include <sys/socket.h>

#include "../../../include/mv2h.h"
#include "internode.h"
#include "log.h"
#include "world.h"
#include "../coll/kernels.h"

namespace mv2 {

namespace {

struct Req {
    bool send;
    bool done = false;
    int err = 0;
    // send
    bool sdev = false;  // sbuf is device memory (chunk copies as kernels)
    bool rdev = false;  // rbuf is device memory
    const char *sbuf = nullptr;
    size_t bytes = 0, off = 0;
    int peer = -1, tag = 0;
    uint64_t msg = 0;
    // receive
    char *rbuf = nullptr;
    size_t cap = 0;
    int src_want = 0, tag_want = 0;
    int src = -1, rtag = -1;
    size_t total = 0;
};

// An unexpected message from a rank of this node keeps its payload in device memory (`dev`, a
// pooled block: arena -> block -> the receive's buffer, never through the host); one from the rank
// mesh, or when no device block can be had, in host memory (`data`).
struct Unexp {
    int src, tag;
    size_t total;
    size_t got = 0;  // bytes landed in `dev` / `data` (copies synchronised)
    bool complete = false;
    std::vector<char> data;
    char *dev = nullptr;
    ~Unexp() {
        if (dev) pool_put(dev);
    }
};

// message currently arriving on the channel from one source
struct Arrival {
    bool active = false;
    size_t total = 0, got = 0;  // got: chunks issued (bytes)
    Req *req = nullptr;         // matched receive, or
    Unexp *ux = nullptr;        // unexpected buffer
};

std::unordered_map<uint64_t, Req *> g_reqs;
uint64_t g_next_id = 1;
uint64_t g_msg_seq = 0;
std::deque<Req *> g_sendq[kMaxRanks];  // per destination, FIFO (one message at a time per channel)
std::list<Req *> g_posted;             // unmatched receives in posting order
std::list<Unexp *> g_unexp;            // unexpected messages in arrival order
uint64_t g_unexp_matched = 0;          // unexpected messages later taken by a receive (mv2h_get_info)
Arrival g_in[kMaxRanks];

// rank mesh (ranks on other nodes)
struct NetHdr {
    int32_t magic;
    int32_t src;  // sender's global rank
    int32_t tag;
    int32_t pad;
    uint64_t bytes;
};
constexpr int32_t kNetMagic = 0x6d763270;  // "mv2p"
struct NetOut {
    Req *r;
    std::vector<char> buf;  // header + payload (staged to host at MPI_Isend)
    size_t off;
};
struct NetIn {
    NetHdr hdr;
    size_t hgot = 0;
    bool body = false;
    std::vector<char> stage;  // the payload, host
    size_t got = 0;
    Req *req = nullptr;    // matched receive, or
    Unexp *ux = nullptr;   // unexpected message (filled when the payload is complete)
};
std::deque<NetOut> g_netq[kMeshMaxRanks];
NetIn g_netin[kMeshMaxRanks];

int node_base() { return world().node * world().size; }
bool on_node(int g) { return g >= node_base() && g < node_base() + world().size; }

bool matches(const Req *r, int src, int tag) {
    // MPI_ANY_TAG matches application tags only (>= 0), never the library's collective context
    return (r->src_want == MV2H_ANY_SOURCE || r->src_want == src) &&
           (r->tag_want == tag || (r->tag_want == MV2H_ANY_TAG && tag >= 0));
}

char *slot_ptr(char *arena, int src, uint64_t pos) {
    return arena + ((size_t)src * kP2PSlots + (size_t)(pos % kP2PSlots)) * kP2PChunk;
}

// Chunk copies between device buffers and the arenas run as copy kernels (coll/kernels.h
// launch_pack_strided, one contiguous row), the last of a progress pass raising a completion word
// of the point-to-point stream's own (counters + pinned host word, separate from the collectives'
// one: a nonblocking collective may be in flight on the library stream meanwhile).  hipMemcpyAsync
// plus hipStreamSynchronize cost 26 us per message below 32 KiB and 53-58 us from 32 KiB to
// 8 MiB on the shared MI355X (profiles/r05f: SDMA or blit engines alike), the kernels 17 / 22-26 us
// (r05g).  With more than four ranks on one GPU the copy engines stay: eight processes' copy
// kernels contending for the shared GPU's compute queues made the user-op line's all-to-all of
// 2 MiB ranges 2.4x slower (C-op line at 8 shared ranks 18.1 ms with kernels, 7.5 ms on the
// engines: r05j / r05l), while at 4 shared ranks the kernels still win (5.0 vs 5.4 ms; osu_bw pattern
// 442 vs 145 GB/s: r05i / r05l).  Host buffers and the unexpected-message buffers keep
// hipMemcpyAsync.  MV2AMD_P2P_KERNEL_COPY=0 / 1 forces either.
struct P2PDone {
    uint32_t *ctr = nullptr;
    uint64_t *flag = nullptr;
    uint64_t seq = 0;
};
P2PDone g_pdone;
bool g_kcopy = true;

int ready() {
    World &w = world();
    if (!w.inited || !w.p2p || (w.size > 1 && !w.shm)) {
        MV2_ERR("point-to-point needs MPI_Init and at most %d ranks on the node", kMaxRanks);
        return E_OTHER;
    }
    // created on first use: an idle extra stream still costs a hardware queue, and
    // collective-only jobs (several ranks sharing a GPU in tests) measured slower with it
    if (!w.p2p_stream) {
        if (hipStreamCreate(&w.p2p_stream) != hipSuccess) return E_OTHER;
        const char *v = getenv("MV2AMD_P2P_KERNEL_COPY");
        g_kcopy = (v && *v) ? *v != '0' : w.nshare <= 4;
        if (g_kcopy && (hipMalloc((void **)&g_pdone.ctr, kDoneBytes) != hipSuccess ||
                        hipMemset(g_pdone.ctr, 0, kDoneBytes) != hipSuccess ||
                        hipHostMalloc((void **)&g_pdone.flag, 64, hipHostMallocDefault) != hipSuccess)) {
            (void)hipGetLastError();
            g_kcopy = false;  // the copy engines then (hipMemcpyAsync + stream synchronisation)
        }
        if (g_pdone.flag) memset(g_pdone.flag, 0, 64);
        if (g_kcopy) hipDeviceSynchronize();
    }
    return 0;
}

bool dev_ptr(const void *p) {
    hipPointerAttribute_t a;
    if (!p || hipPointerGetAttributes(&a, p) != hipSuccess) {
        (void)hipGetLastError();
        return false;
    }
    return a.type == hipMemoryTypeDevice;
}

// one chunk copy of a progress pass
struct Copy {
    char *dst;
    const char *src;
    size_t len;
    bool kernel;  // both sides device memory: a copy kernel
};

// Issue a pass's copies on the point-to-point stream and wait for all of them: a completion word
// when the pass ends in a copy kernel, else a stream synchronisation.
int run_copies(const std::vector<Copy> &cp) {
    World &w = world();
    const hipStream_t st = w.p2p_stream;
    for (size_t i = 0; i < cp.size(); ++i) {
        const Copy &c = cp[i];
        if (!c.len) continue;
        if (c.kernel) {
            // every copy kernel carries the word (the host waits for the last value only): its
            // completion writes back the L2 of each XCD its workgroups ran on.  A kernel without it
            // left dirty lines in the L2s the next, smaller kernel's write-back did not reach
            // (block_done flushes the XCDs of its own workgroups), and a receiver on this node read
            // the arena slot stale there (r05al: 3-5 blocks of 64 KiB of a 4 MiB operand)
            const Done d{g_pdone.ctr, g_pdone.flag, ++g_pdone.seq};
            if (launch_pack_strided(c.src, c.dst, 1, c.len, c.len, 0, st, d) != 0) {
                MV2_ERR("point-to-point copy kernel failed to launch: %s", hipGetErrorString(hipGetLastError()));
                return E_INTERN;
            }
        } else if (hipMemcpyAsync(c.dst, c.src, c.len, hipMemcpyDefault, st) != hipSuccess) {
            MV2_ERR("point-to-point chunk copy failed: %s", hipGetErrorString(hipGetLastError()));
            return E_INTERN;
        }
    }
    // the word alone proves the pass complete only when every copy of it is a kernel: a host
    // buffer's hipMemcpyAsync may finish (staged through pinned memory) after the kernels behind it
    bool all_kernels = true;
    for (const Copy &c : cp) all_kernels = all_kernels && (c.kernel || !c.len);
    const bool word = all_kernels && !cp.empty() && cp.back().kernel && cp.back().len;
    if (word) {
        // the word is the normal path; the stream is consulted once it is 200 us late, then every 100 us
        const uint64_t want = g_pdone.seq;
        auto t0 = std::chrono::steady_clock::now();
        double next_us = 200.0;
        // a word raised by a copy kernel whose block groups ran on several XCDs (device_util.h
        // block_done): done once the stream is, as for the collectives (coll.cpp settle_split)
        auto settle = [&]() {
            static uint64_t seen = 0;
            const uint64_t s = __atomic_load_n(g_pdone.flag + 1, __ATOMIC_ACQUIRE);
            if (s <= seen) return 0;
            seen = s;
            ++w.done_xcd_split;
            return hipStreamSynchronize(st) == hipSuccess ? 0 : E_INTERN;
        };
        bool queried = false;
        for (unsigned spins = 0;; ++spins) {
            if (__atomic_load_n(g_pdone.flag, __ATOMIC_ACQUIRE) >= want) return settle();
            if ((spins & 255u) != 0) continue;
            const double us = std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count();
            if (us < next_us) continue;
            next_us = us + 100.0;
            if (!queried) {
                queried = true;
                ++w.done_queried;
            }
            const hipError_t q = hipStreamQuery(st);
            if (q == hipErrorNotReady) continue;
            if (__atomic_load_n(g_pdone.flag, __ATOMIC_ACQUIRE) >= want) {
                if (q == hipSuccess) ++w.done_late;
                return settle();
            }
            if (q == hipSuccess) {  // finished without raising the word: counters reset, done
                if (w.done_missed++ == 0)
                    fprintf(stderr, "[mv2amd rank %d] warning: a point-to-point copy kernel finished without raising "
                                    "its completion word; completing by stream synchronisation (counted in done_missed)\n",
                            log_rank());
                hipMemsetAsync(g_pdone.ctr, 0, kDoneBytes, st);
                return hipStreamSynchronize(st) == hipSuccess ? 0 : E_INTERN;
            }
            MV2_ERR("point-to-point copies failed: %s", hipGetErrorString(q));
            return E_INTERN;
        }
    }
    if (hipStreamSynchronize(st) != hipSuccess) {
        MV2_ERR("point-to-point copies failed: %s", hipGetErrorString(hipGetLastError()));
        return E_INTERN;
    }
    return 0;
}

// a header from global rank src: the receive it matches (posting order), else an unexpected
// message; the payload lands in `stage` and is delivered when complete
void net_header(NetIn &in, int src) {
    in.req = nullptr;
    in.ux = nullptr;
    for (auto it = g_posted.begin(); it != g_posted.end(); ++it) {
        if (matches(*it, src, in.hdr.tag)) {
            in.req = *it;
            g_posted.erase(it);
            break;
        }
    }
    if (in.req) {
        in.req->src = src;
        in.req->rtag = in.hdr.tag;
        in.req->total = in.hdr.bytes;
    } else {
        in.ux = new Unexp{src, in.hdr.tag, (size_t)in.hdr.bytes};
        g_unexp.push_back(in.ux);
    }
    in.stage.resize(in.hdr.bytes);
    in.got = 0;
    in.body = true;
}

int net_deliver(NetIn &in) {
    in.body = false;
    in.hgot = 0;
    if (in.req) {
        Req *r = in.req;
        const size_t n = std::min(r->total, r->cap);
        if (n) {  // complete (stream-synchronised) before the receive is
            const std::vector<Copy> one{{r->rbuf, in.stage.data(), n, false}};
            if (const int rc = run_copies(one)) return rc;
        }
        if (r->total > r->cap) r->err = E_TRUNCATE;
        r->done = true;
    } else if (in.ux) {
        in.ux->data.swap(in.stage);
        if (in.ux->data.empty()) in.ux->data.resize(1);
        in.ux->got = in.ux->total;
        in.ux->complete = true;
    }
    in.req = nullptr;
    in.ux = nullptr;
    in.stage.clear();
    return 0;
}

// non-blocking pass over the rank mesh: write queued messages, read headers and payloads
int net_progress(bool *moved) {
    World &w = world();
    if (w.nnodes <= 1) return 0;
    for (int g = 0; g < w.gsize && g < kMeshMaxRanks; ++g) {
        const int fd = mesh_fd(g);
        if (fd < 0) continue;
        while (!g_netq[g].empty()) {
            NetOut &o = g_netq[g].front();
            const ssize_t k = send(fd, o.buf.data() + o.off, o.buf.size() - o.off, MSG_DONTWAIT | MSG_NOSIGNAL);
            if (k < 0) {
                if (errno == EAGAIN || errno == EWOULDBLOCK || errno == EINTR) break;
                MV2_ERR("point-to-point to rank %d (rank mesh): send failed: %s", g, strerror(errno));
                return E_OTHER;
            }
            o.off += (size_t)k;
            *moved = *moved || k > 0;
            if (o.off < o.buf.size()) break;
            o.r->done = true;
            g_netq[g].pop_front();
        }
        NetIn &in = g_netin[g];
        for (;;) {
            char *dst;
            size_t want;
            if (!in.body) {
                dst = (char *)&in.hdr + in.hgot;
                want = sizeof(NetHdr) - in.hgot;
            } else {
                dst = in.stage.data() + in.got;
                want = in.stage.size() - in.got;
            }
            if (want) {
                const ssize_t k = recv(fd, dst, want, MSG_DONTWAIT);
                if (k == 0) {
                    MV2_ERR("point-to-point from rank %d (rank mesh): connection closed by the peer (%s): that rank "
                            "has exited", g, in.body ? "inside a message" : "between messages");
                    return E_OTHER;
                }
                if (k < 0) {
                    if (errno == EAGAIN || errno == EWOULDBLOCK || errno == EINTR) break;
                    MV2_ERR("point-to-point from rank %d (rank mesh): recv failed: %s", g, strerror(errno));
                    return E_OTHER;
                }
                *moved = true;
                if (!in.body) in.hgot += (size_t)k;
                else in.got += (size_t)k;
                if ((!in.body && in.hgot < sizeof(NetHdr)) || (in.body && in.got < in.stage.size())) continue;
            }
            if (!in.body) {
                if (in.hdr.magic != kNetMagic || in.hdr.src != g) {
                    MV2_ERR("point-to-point from rank %d: stream out of sequence", g);
                    return E_INTERN;
                }
                net_header(in, g);
                if (in.stage.empty()) {  // empty message: complete at its header
                    const int rc = net_deliver(in);
                    if (rc) return rc;
                }
            } else {
                const int rc = net_deliver(in);
                if (rc) return rc;
            }
        }
    }
    return 0;
}

// One progress pass: push queued send chunks into free slots, drain arrived
// chunks into matched receives / unexpected buffers.  Returns an error class
// or 0; *moved = whether anything happened.
int progress(bool *moved) {
    World &w = world();
    const int n = w.size, me = w.rank;
    *moved = false;

    struct SendPub {
        P2PChan *c;
        uint64_t pos;
        P2PRec rec;
        Req *r;
        bool last;
    };
    struct RecvPub {
        P2PChan *c;
        uint64_t head;  // new head after this chunk
        int src;
        size_t len;
        bool last;
        Req *r;
        Unexp *ux;
    };
    std::vector<SendPub> sp;
    std::vector<RecvPub> rp;
    std::vector<Copy> cp;
    const int base = node_base();
    if (!w.shm) return net_progress(moved);

    for (int d = 0; d < n; ++d) {
        if (g_sendq[d].empty()) continue;
        P2PChan &c = w.shm->chan[me][d];
        uint64_t tail = c.tail.load(std::memory_order_relaxed);
        const uint64_t head = c.head.load(std::memory_order_acquire);
        while (!g_sendq[d].empty() && tail - head < (uint64_t)kP2PSlots) {
            Req *r = g_sendq[d].front();
            const size_t len = std::min(kP2PChunk, r->bytes - r->off);
            if (len) cp.push_back({slot_ptr(w.peer_p2p[d], me, tail), r->sbuf + r->off, len, g_kcopy && r->sdev});
            P2PRec rec{r->msg, r->tag, 0, r->bytes, r->off, len};
            r->off += len;
            const bool last = r->off >= r->bytes;
            sp.push_back({&c, tail, rec, r, last});
            ++tail;
            if (last) g_sendq[d].pop_front();
        }
    }

    for (int s = 0; s < n; ++s) {
        P2PChan &c = w.shm->chan[s][me];
        uint64_t head = c.head.load(std::memory_order_relaxed);
        const uint64_t tail = c.tail.load(std::memory_order_acquire);
        Arrival &a = g_in[s];
        while (head < tail) {
            const P2PRec rec = c.rec[head % kP2PSlots];
            if (!a.active) {
                if (rec.off != 0) {
                    MV2_ERR("point-to-point channel from rank %d out of sequence", s);
                    return E_INTERN;
                }
                a = Arrival{};
                a.active = true;
                a.total = rec.total;
                for (auto it = g_posted.begin(); it != g_posted.end(); ++it) {
                    if (matches(*it, base + s, rec.tag)) {
                        a.req = *it;
                        g_posted.erase(it);
                        break;
                    }
                }
                if (a.req) {
                    a.req->src = base + s;
                    a.req->rtag = rec.tag;
                    a.req->total = rec.total;
                } else {
                    a.ux = new Unexp{base + s, rec.tag, (size_t)rec.total};
                    if (!(a.ux->dev = rec.total ? (char *)pool_get((size_t)rec.total) : nullptr))
                        a.ux->data.resize(rec.total ? rec.total : 1);
                    g_unexp.push_back(a.ux);
                }
            }
            const char *src = slot_ptr(w.p2p, s, head);
            if (a.req) {
                const size_t room = a.req->cap > rec.off ? std::min<size_t>(rec.len, a.req->cap - rec.off) : 0;
                if (room) cp.push_back({a.req->rbuf + rec.off, src, room, g_kcopy && a.req->rdev});
            } else if (rec.len) {
                if (a.ux->dev) cp.push_back({a.ux->dev + rec.off, src, (size_t)rec.len, g_kcopy});
                else cp.push_back({a.ux->data.data() + rec.off, src, (size_t)rec.len, false});
            }
            a.got += rec.len;
            ++head;
            const bool last = a.got >= a.total;
            rp.push_back({&c, head, s, (size_t)rec.len, last, a.req, a.ux});
            if (last) a.active = false;
        }
    }

    int rc = net_progress(moved);
    if (rc) return rc;
    if (sp.empty() && rp.empty()) return 0;
    *moved = true;
    if ((rc = run_copies(cp))) return rc;
    // data is in place: publish records / free slots, complete requests
    for (const SendPub &p : sp) {
        p.c->rec[p.pos % kP2PSlots] = p.rec;
        p.c->tail.store(p.pos + 1, std::memory_order_release);
        if (p.last) p.r->done = true;
    }
    for (const RecvPub &p : rp) {
        p.c->head.store(p.head, std::memory_order_release);
        if (p.ux) {
            p.ux->got += p.len;
            if (p.last) p.ux->complete = true;
        }
        if (p.r && p.last) {
            if (p.r->total > p.r->cap) p.r->err = E_TRUNCATE;
            p.r->done = true;
        }
    }
    return 0;
}

bool g_coll_poisoned = false;  // a collective gave up a request mid-flight (p2p_abandon)

int coll_context_check(int tag) {
    if (tag <= kCollTagBase && g_coll_poisoned) {
        MV2_ERR("an earlier collective failed with a message in flight: the library's collective context is "
                "unusable (MPI_ERR_OTHER for every later collective that sends or receives)");
        return E_OTHER;
    }
    return 0;
}

uint64_t add_req(Req *r) {
    const uint64_t id = g_next_id++;
    g_reqs[id] = r;
    return id;
}

}  // namespace
}  // namespace mv2

using namespace mv2;

int mv2::p2p_isend(const void *buf, size_t bytes, int dest, int tag, unsigned long long *req) {
    int rc = ready();
    if (rc || (rc = coll_context_check(tag))) return rc;
    World &w = world();
    if (dest < 0 || dest >= w.gsize) return E_RANK;
    if (bytes && !buf) return E_BUFFER;
    Req *r = new Req{};
    r->send = true;
    r->sbuf = (const char *)buf;
    r->sdev = g_kcopy && dev_ptr(buf);
    r->bytes = bytes;
    r->peer = dest;
    r->tag = tag;
    r->msg = ++g_msg_seq;
    if (!on_node(dest)) {  // rank mesh: header + payload staged to host now, written by progress
        if (mesh_fd(dest) < 0) {
            delete r;
            MV2_ERR("no point-to-point link to rank %d on another node (jobs up to %d ranks)", dest, kMeshMaxRanks);
            return E_UNSUPPORTED;
        }
        NetOut o{r, std::vector<char>(sizeof(NetHdr) + bytes), 0};
        const NetHdr h{kNetMagic, w.grank, tag, 0, (uint64_t)bytes};
        memcpy(o.buf.data(), &h, sizeof(h));
        if (bytes && hipMemcpy(o.buf.data() + sizeof(h), buf, bytes, hipMemcpyDefault) != hipSuccess) {
            delete r;
            return E_INTERN;
        }
        g_netq[dest].push_back(std::move(o));
        *req = add_req(r);
        bool moved = false;
        return net_progress(&moved);
    }
    if (!w.shm) {  // a node of one rank sending to itself: matched and delivered right here
        NetIn in;
        in.hdr = NetHdr{kNetMagic, w.grank, tag, 0, (uint64_t)bytes};
        net_header(in, w.grank);
        if (bytes && hipMemcpy(in.stage.data(), buf, bytes, hipMemcpyDefault) != hipSuccess) {
            delete r;
            return E_INTERN;
        }
        if ((rc = net_deliver(in))) {
            delete r;
            return rc;
        }
        r->done = true;
        *req = add_req(r);
        return 0;
    }
    g_sendq[dest - node_base()].push_back(r);
    *req = add_req(r);
    bool moved;
    return progress(&moved);  // eager: start pushing right away
}

int mv2::p2p_irecv(void *buf, size_t cap, int source, int tag, unsigned long long *req) {
    int rc = ready();
    if (rc || (rc = coll_context_check(tag))) return rc;
    World &w = world();
    if (source != MV2H_ANY_SOURCE && (source < 0 || source >= w.gsize)) return E_RANK;
    if (cap && !buf) return E_BUFFER;
    Req *r = new Req{};
    r->send = false;
    r->rbuf = (char *)buf;
    r->rdev = g_kcopy && dev_ptr(buf);
    r->cap = cap;
    r->src_want = source;
    r->tag_want = tag;
    *req = add_req(r);
    // earliest matching unexpected message first (arrival order)
    for (auto it = g_unexp.begin(); it != g_unexp.end(); ++it) {
        Unexp *u = *it;
        if (!matches(r, u->src, u->tag)) continue;
        ++g_unexp_matched;
        r->src = u->src;
        r->rtag = u->tag;
        r->total = u->total;
        const size_t have = std::min(u->got, cap);
        if (have) {  // complete before the receive can be: the caller may read buf on any stream next
            const std::vector<Copy> one{{(char *)buf, u->dev ? u->dev : u->data.data(), have, u->dev && r->rdev}};
            if ((rc = run_copies(one))) return rc;
        }
        g_unexp.erase(it);
        if (u->complete) {
            if (u->total > cap) r->err = E_TRUNCATE;
            r->done = true;
        } else if (!on_node(u->src)) {
            // still arriving on the rank mesh: the payload goes to this receive when complete
            NetIn &in = g_netin[u->src];
            in.ux = nullptr;
            in.req = r;
        } else {
            // still arriving: the rest of its chunks go straight to the user buffer
            Arrival &a = g_in[u->src - node_base()];
            a.ux = nullptr;
            a.req = r;
        }
        delete u;
        bool moved;
        return progress(&moved);
    }
    g_posted.push_back(r);
    bool moved;
    return progress(&moved);
}

bool mv2::coll_context_poisoned() { return g_coll_poisoned; }
unsigned long long mv2::p2p_unexpected_matched() { return g_unexp_matched; }

void mv2::p2p_abandon(unsigned long long id) {
    auto it = g_reqs.find(id);
    if (it == g_reqs.end()) return;
    Req *r = it->second;
    const auto pit = std::find(g_posted.begin(), g_posted.end(), r);
    if (pit != g_posted.end() || r->done) {  // never matched (or finished): nothing refers to it
        if (pit != g_posted.end()) g_posted.erase(pit);
        g_reqs.erase(it);
        delete r;
        return;
    }
    // matched and still arriving, or a send still queued: the transport keeps referring to it, so
    // it stays allocated, and later collectives refuse to run rather than match what follows
    g_coll_poisoned = true;
}

extern "C" {

int mv2h_isend(const void *buf, size_t bytes, int dest, int tag, unsigned long long *req) {
    if (tag < 0) return E_TAG;
    return p2p_isend(buf, bytes, dest, tag, req);
}

int mv2h_irecv(void *buf, size_t cap, int source, int tag, unsigned long long *req) {
    if (tag < 0 && tag != MV2H_ANY_TAG) return E_TAG;
    return p2p_irecv(buf, cap, source, tag, req);
}

int mv2h_p2p_test(unsigned long long id, int *done, int *source, int *tag, size_t *bytes) {
    auto it = g_reqs.find(id);
    if (it == g_reqs.end()) return E_REQUEST;
    Req *r = it->second;
    if (!r->done) {
        bool moved;
        const int rc = progress(&moved);
        if (rc) return rc;
    }
    *done = r->done ? 1 : 0;
    if (!r->done) return 0;
    if (!r->send) {
        if (source) *source = r->src;
        if (tag) *tag = r->rtag;
        if (bytes) *bytes = std::min(r->total, r->cap);
    }
    const int err = r->err;
    g_reqs.erase(it);
    delete r;
    return err;
}

int mv2h_p2p_peek(unsigned long long id, int *done) {
    auto it = g_reqs.find(id);
    if (it == g_reqs.end()) return E_REQUEST;
    if (!it->second->done) {
        bool moved;
        const int rc = progress(&moved);
        if (rc) return rc;
    }
    *done = it->second->done ? 1 : 0;
    return 0;
}

int mv2h_p2p_wait(unsigned long long id, int *source, int *tag, size_t *bytes) {
    if (g_reqs.find(id) == g_reqs.end()) return E_REQUEST;
    beacon(BC_P2P_WAIT);
    const auto t0 = std::chrono::steady_clock::now();
    const char *tv = getenv("MV2AMD_TIMEOUT_S");
    const double limit = (tv && *tv) ? atof(tv) : 120.0;
    unsigned idle = 0;
    for (;;) {
        int done = 0;
        const int rc = mv2h_p2p_test(id, &done, source, tag, bytes);
        if (done || rc) return rc;
        if (++idle > 64) {
            sched_yield();
            if ((idle & 1023) == 0 &&
                std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count() > limit) {
                MV2_ERR("point-to-point request not matched within %.0f s (MV2AMD_TIMEOUT_S)", limit);
                return E_OTHER;
            }
        }
    }
}

int mv2h_p2p_progress(void) {
    if (ready()) return 0;
    bool moved;
    return progress(&moved);
}

}  // extern "C"
