// internode.cpp — leader transport between nodes (internode.h).
//
// The reference's two-level collectives run their inter-node step on leader_comm, the
// communicator of the nodes' local rank 0 (create_2level_comm.c:1843), over its network
// channel.  Here the leaders keep one TCP stream per pair of nodes:
//   rendezvous: the leader of node 0 listens on MV2AMD_BOOT_ADDR:MV2AMD_BOOT_PORT (default
//               MASTER_ADDR : MASTER_PORT + 1); every other leader opens its own listener,
//               connects, and sends {node, listener port}; node 0 answers with every
//               leader's address and port (the boot connections stay as the links to node 0);
//   mesh:       leader i connects to leaders 1 .. i-1 and accepts leaders i+1 .. n-1.
// Every exchange is a fixed-size message both sides know in advance (the schedules of the
// collectives are deterministic), so there is no framing; sendrecv interleaves both
// directions with poll() so two leaders exchanging large buffers never block each other.
#include "internode.h"

#include <arpa/inet.h>
#include <errno.h>
#include <netdb.h>
#include <netinet/in.h>
#include <netinet/tcp.h>
#include <poll.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <sys/socket.h>
#include <time.h>
#include <unistd.h>

#include <string>
#include <vector>

#include "../common.h"
#include "log.h"
#include "world.h"

namespace mv2 {

namespace {

struct Hello {
    int32_t magic;
    int32_t node;
    int32_t port;  // the sender's mesh listener
    int32_t nnodes;
    int32_t ppn;         // ranks per node (the schedules assume the same count everywhere)
    int32_t pad;
    uint64_t knob_hash;  // FNV-1a of the MV2_* selection knobs (every node must select alike)
};

uint64_t knob_hash() {
    const unsigned char *p = (const unsigned char *)&knobs();
    uint64_t h = 1469598103934665603ull;
    for (size_t i = 0; i < sizeof(Knobs); ++i) h = (h ^ p[i]) * 1099511628211ull;
    return h;
}
struct Entry {
    char ip[64];
    int32_t port;
};
constexpr int32_t kMagic = 0x6d76326e;  // "mv2n"

struct Net {
    std::vector<int> fd;  // fd[node] (-1: self / not connected)
    int listen_fd = -1;
    bool up = false;
    std::vector<std::string> ip;  // every node's address (the rendezvous' view; node 0: the boot host)
};
Net g_net;

// rank mesh: one TCP stream between every pair of ranks on different nodes (point-to-point
// across nodes, runtime/p2p.cpp)
struct Mesh {
    std::vector<int> fd;  // fd[global rank] (-1: same node / not connected)
    int listen_fd = -1;
};
Mesh g_mesh;
struct MeshHello {
    int32_t magic;
    int32_t grank;
};

double now_s() {
    timespec t;
    clock_gettime(CLOCK_MONOTONIC, &t);
    return (double)t.tv_sec + 1e-9 * (double)t.tv_nsec;
}

double timeout_s() {
    const char *v = getenv("MV2AMD_TIMEOUT_S");
    const long t = v && *v ? atol(v) : 120;
    return t > 0 ? (double)t : 120.0;
}

void tune(int fd) {
    int one = 1;
    setsockopt(fd, IPPROTO_TCP, TCP_NODELAY, &one, sizeof(one));
    int buf = 8 << 20;
    setsockopt(fd, SOL_SOCKET, SO_SNDBUF, &buf, sizeof(buf));
    setsockopt(fd, SOL_SOCKET, SO_RCVBUF, &buf, sizeof(buf));
}

int open_listener(const char *addr, int port, int *bound_port) {
    const int fd = socket(AF_INET, SOCK_STREAM, 0);
    if (fd < 0) return -1;
    int one = 1;
    setsockopt(fd, SOL_SOCKET, SO_REUSEADDR, &one, sizeof(one));
    sockaddr_in sa{};
    sa.sin_family = AF_INET;
    sa.sin_port = htons((uint16_t)port);
    sa.sin_addr.s_addr = addr ? inet_addr(addr) : htonl(INADDR_ANY);
    if (bind(fd, (sockaddr *)&sa, sizeof(sa)) != 0 || listen(fd, 64) != 0) {
        close(fd);
        return -1;
    }
    socklen_t len = sizeof(sa);
    getsockname(fd, (sockaddr *)&sa, &len);
    if (bound_port) *bound_port = ntohs(sa.sin_port);
    return fd;
}

int connect_retry(const char *host, int port) {
    const double t_end = now_s() + timeout_s();
    addrinfo hints{}, *res = nullptr;
    hints.ai_family = AF_INET;
    hints.ai_socktype = SOCK_STREAM;
    char ps[16];
    snprintf(ps, sizeof(ps), "%d", port);
    if (getaddrinfo(host, ps, &hints, &res) != 0 || !res) return -1;
    int fd = -1;
    while (now_s() < t_end) {
        fd = socket(AF_INET, SOCK_STREAM, 0);
        if (fd < 0) break;
        if (connect(fd, res->ai_addr, res->ai_addrlen) == 0) break;
        close(fd);
        fd = -1;
        usleep(20000);  // the peer's listener is not up yet
    }
    freeaddrinfo(res);
    if (fd >= 0) tune(fd);
    return fd;
}

// a host name or address as dotted IPv4 (the form every node's ranks connect to, and what fits the
// control segment's node_ip); "" when it does not resolve
std::string numeric_ipv4(const std::string &host) {
    addrinfo hints{}, *res = nullptr;
    hints.ai_family = AF_INET;
    hints.ai_socktype = SOCK_STREAM;
    if (getaddrinfo(host.c_str(), nullptr, &hints, &res) != 0 || !res) return "";
    char buf[INET_ADDRSTRLEN] = {};
    inet_ntop(AF_INET, &((const sockaddr_in *)res->ai_addr)->sin_addr, buf, sizeof(buf));
    freeaddrinfo(res);
    return buf;
}

int accept_timed(int lfd) {
    pollfd p{lfd, POLLIN, 0};
    const int ms = (int)(timeout_s() * 1000.0);
    if (poll(&p, 1, ms) <= 0) return -1;
    const int fd = accept(lfd, nullptr, nullptr);
    if (fd >= 0) tune(fd);
    return fd;
}

// full-duplex transfer on one socket: send sn bytes and receive rn bytes, interleaved.  `peer`
// names the other end in the diagnostics (a node index on the leaders' links, -1: bootstrap);
// every failure path says what failed, with errno, before the caller closes anything.
int xfer(int fd, const char *sb, size_t sn, char *rb, size_t rn, int peer = -1) {
    size_t so = 0, ro = 0;
    const int ms = (int)(timeout_s() * 1000.0);
    while (so < sn || ro < rn) {
        pollfd p{fd, (short)((so < sn ? POLLOUT : 0) | (ro < rn ? POLLIN : 0)), 0};
        const int r = poll(&p, 1, ms);
        if (r <= 0) {
            if (r < 0 && errno == EINTR) continue;
            if (r < 0) MV2_ERR("inter-node link to node %d: poll failed: %s", peer, strerror(errno));
            else MV2_ERR("inter-node link to node %d: no progress for %.0f s (MV2AMD_TIMEOUT_S; sent %zu of %zu, "
                         "received %zu of %zu bytes)", peer, timeout_s(), so, sn, ro, rn);
            return E_OTHER;
        }
        if (p.revents & (POLLERR | POLLHUP | POLLNVAL) && !(p.revents & POLLIN)) {
            MV2_ERR("inter-node link to node %d lost (poll revents 0x%x; sent %zu of %zu, received %zu of %zu bytes)",
                    peer, (unsigned)p.revents, so, sn, ro, rn);
            return E_OTHER;
        }
        if ((p.revents & POLLIN) && ro < rn) {
            const ssize_t k = recv(fd, rb + ro, rn - ro, 0);
            if (k == 0) {
                MV2_ERR("inter-node link to node %d closed by the peer (received %zu of %zu bytes): that node's "
                        "leader has exited", peer, ro, rn);
                return E_OTHER;
            }
            if (k < 0 && errno != EINTR && errno != EAGAIN) {
                MV2_ERR("inter-node link to node %d: recv failed: %s", peer, strerror(errno));
                return E_OTHER;
            }
            if (k > 0) ro += (size_t)k;
        }
        if ((p.revents & POLLOUT) && so < sn) {
            const ssize_t k = send(fd, sb + so, sn - so, MSG_NOSIGNAL | MSG_DONTWAIT);
            if (k < 0 && errno != EINTR && errno != EAGAIN && errno != EWOULDBLOCK) {
                MV2_ERR("inter-node link to node %d: send failed: %s", peer, strerror(errno));
                return E_OTHER;
            }
            if (k > 0) so += (size_t)k;
        }
    }
    return 0;
}

// send sn bytes on fd_out while receiving rn bytes on fd_in (a ring step: different peers),
// interleaved so that neither side's socket buffers can fill up and stall the ring
int xfer2(int fd_out, const char *sb, size_t sn, int fd_in, char *rb, size_t rn, int to, int from) {
    size_t so = 0, ro = 0;
    const int ms = (int)(timeout_s() * 1000.0);
    while (so < sn || ro < rn) {
        pollfd p[2] = {{fd_out, (short)(so < sn ? POLLOUT : 0), 0}, {fd_in, (short)(ro < rn ? POLLIN : 0), 0}};
        const int r = poll(p, 2, ms);
        if (r <= 0) {
            if (r < 0 && errno == EINTR) continue;
            if (r < 0) MV2_ERR("inter-node ring step (to node %d, from node %d): poll failed: %s", to, from, strerror(errno));
            else MV2_ERR("inter-node ring step (to node %d, from node %d): no progress for %.0f s (MV2AMD_TIMEOUT_S; "
                         "sent %zu of %zu, received %zu of %zu bytes)", to, from, timeout_s(), so, sn, ro, rn);
            return E_OTHER;
        }
        if ((p[1].revents & POLLIN) && ro < rn) {
            const ssize_t k = recv(fd_in, rb + ro, rn - ro, 0);
            if (k == 0) {
                MV2_ERR("inter-node link from node %d closed by the peer (received %zu of %zu bytes): that node's "
                        "leader has exited", from, ro, rn);
                return E_OTHER;
            }
            if (k < 0 && errno != EINTR && errno != EAGAIN) {
                MV2_ERR("inter-node link from node %d: recv failed: %s", from, strerror(errno));
                return E_OTHER;
            }
            if (k > 0) ro += (size_t)k;
        } else if (p[1].revents & (POLLERR | POLLHUP | POLLNVAL)) {
            MV2_ERR("inter-node link from node %d lost (poll revents 0x%x)", from, (unsigned)p[1].revents);
            return E_OTHER;
        }
        if ((p[0].revents & POLLOUT) && so < sn) {
            const ssize_t k = send(fd_out, sb + so, sn - so, MSG_NOSIGNAL | MSG_DONTWAIT);
            if (k < 0 && errno != EINTR && errno != EAGAIN && errno != EWOULDBLOCK) {
                MV2_ERR("inter-node link to node %d: send failed: %s", to, strerror(errno));
                return E_OTHER;
            }
            if (k > 0) so += (size_t)k;
        } else if (p[0].revents & (POLLERR | POLLHUP | POLLNVAL)) {
            MV2_ERR("inter-node link to node %d lost (poll revents 0x%x)", to, (unsigned)p[0].revents);
            return E_OTHER;
        }
    }
    return 0;
}

int link_fd(int peer) {
    if (peer < 0 || peer >= (int)g_net.fd.size() || g_net.fd[peer] < 0) {
        MV2_ERR("no inter-node link to node %d", peer);
        return -1;
    }
    return g_net.fd[peer];
}

}  // namespace

int net_send(int peer, const void *buf, size_t bytes) {
    beacon(BC_NET);
    const int fd = link_fd(peer);
    return fd < 0 ? E_INTERN : xfer(fd, (const char *)buf, bytes, nullptr, 0, peer);
}
int net_recv(int peer, void *buf, size_t bytes) {
    beacon(BC_NET);
    const int fd = link_fd(peer);
    return fd < 0 ? E_INTERN : xfer(fd, nullptr, 0, (char *)buf, bytes, peer);
}
int net_sendrecv(int peer, const void *sbuf, size_t sbytes, void *rbuf, size_t rbytes) {
    beacon(BC_NET);
    const int fd = link_fd(peer);
    return fd < 0 ? E_INTERN : xfer(fd, (const char *)sbuf, sbytes, (char *)rbuf, rbytes, peer);
}

int net_shift(int to, const void *sbuf, size_t sbytes, int from, void *rbuf, size_t rbytes) {
    beacon(BC_NET);
    if (to == from) return net_sendrecv(to, sbuf, sbytes, rbuf, rbytes);
    const int fo = link_fd(to), fi = link_fd(from);
    return fo < 0 || fi < 0 ? E_INTERN : xfer2(fo, (const char *)sbuf, sbytes, fi, (char *)rbuf, rbytes, to, from);
}

int net_init() {
    World &w = world();
    const int nn = w.nnodes, me = w.node;
    g_net.fd.assign((size_t)nn, -1);
    const char *ba = getenv("MV2AMD_BOOT_ADDR");
    const char *ma = getenv("MASTER_ADDR");
    const std::string name = ba && *ba ? ba : (ma && *ma ? ma : "127.0.0.1");
    const std::string host = numeric_ipv4(name);
    if (host.empty()) {
        MV2_ERR("multi-node job: the leaders' rendezvous host '%s' (MV2AMD_BOOT_ADDR / MASTER_ADDR) does not resolve "
                "to an IPv4 address", name.c_str());
        return E_OTHER;
    }
    const char *bp = getenv("MV2AMD_BOOT_PORT");
    const char *mp = getenv("MASTER_PORT");
    const int port = bp && *bp ? atoi(bp) : (mp && *mp ? atoi(mp) + 1 : 0);
    if (port <= 0) {
        MV2_ERR("multi-node job: set MV2AMD_BOOT_PORT (or MASTER_PORT) for the leaders' rendezvous");
        return E_OTHER;
    }
    std::vector<Entry> table((size_t)nn);
    if (me == 0) {
        int bound = 0;
        g_net.listen_fd = open_listener(nullptr, port, &bound);
        if (g_net.listen_fd < 0) {
            MV2_ERR("leader rendezvous: cannot listen on port %d", port);
            return E_OTHER;
        }
        bool mismatch = false;
        for (int k = 1; k < nn; ++k) {
            const int fd = accept_timed(g_net.listen_fd);
            Hello h{};
            if (fd < 0 || xfer(fd, nullptr, 0, (char *)&h, sizeof(h)) || h.magic != kMagic || h.node <= 0 ||
                h.node >= nn || h.nnodes != nn || g_net.fd[h.node] >= 0) {
                MV2_ERR("leader rendezvous: bad or missing hello (%d of %d leaders)", k - 1, nn - 1);
                if (fd >= 0) close(fd);
                return E_OTHER;
            }
            if (h.ppn != w.size || h.knob_hash != knob_hash()) {
                MV2_ERR("node %d differs from node 0 in %s: the nodes would run different schedules", h.node,
                        h.ppn != w.size ? "ranks per node" : "its MV2_* collective selection knobs");
                mismatch = true;
            }
            sockaddr_in sa{};
            socklen_t len = sizeof(sa);
            getpeername(fd, (sockaddr *)&sa, &len);
            inet_ntop(AF_INET, &sa.sin_addr, table[h.node].ip, sizeof(table[h.node].ip));
            table[h.node].port = h.port;
            g_net.fd[h.node] = fd;
        }
        if (mismatch)  // port -1: every leader refuses the job instead of pairing mismatched schedules
            for (Entry &e : table) e.port = -1;
        for (int j = 1; j < nn; ++j)
            if (xfer(g_net.fd[j], (const char *)table.data(), table.size() * sizeof(Entry), nullptr, 0)) return E_OTHER;
        if (mismatch) return E_OTHER;
        g_net.ip.assign((size_t)nn, host);
        for (int j = 1; j < nn; ++j) g_net.ip[j] = table[j].ip;
    } else {
        int myport = 0;
        g_net.listen_fd = open_listener(nullptr, 0, &myport);
        if (g_net.listen_fd < 0) {
            MV2_ERR("leader of node %d: cannot open its mesh listener: %s", me, strerror(errno));
            return E_OTHER;
        }
        const int fd = connect_retry(host.c_str(), port);
        if (fd < 0) {
            MV2_ERR("leader of node %d: cannot reach the rendezvous %s:%d", me, host.c_str(), port);
            return E_OTHER;
        }
        Hello h{kMagic, me, myport, nn, w.size, 0, knob_hash()};
        if (xfer(fd, (const char *)&h, sizeof(h), nullptr, 0) ||
            xfer(fd, nullptr, 0, (char *)table.data(), table.size() * sizeof(Entry))) {
            close(fd);
            return E_OTHER;
        }
        if (table[0].port == -1) {
            MV2_ERR("leader of node %d: node 0 refused the job (ranks per node or MV2_* knobs differ between nodes)", me);
            close(fd);
            return E_OTHER;
        }
        g_net.fd[0] = fd;
        g_net.ip.assign((size_t)nn, host);
        for (int j = 1; j < nn; ++j) g_net.ip[j] = table[j].ip;
        // mesh among nodes 1..nn-1: connect down, accept up
        for (int j = 1; j < me; ++j) {
            const int c = connect_retry(table[j].ip, table[j].port);
            Hello hj{kMagic, me, myport, nn, w.size, 0, knob_hash()};
            if (c < 0 || xfer(c, (const char *)&hj, sizeof(hj), nullptr, 0)) {
                MV2_ERR("leader of node %d: cannot connect to node %d", me, j);
                return E_OTHER;
            }
            g_net.fd[j] = c;
        }
        for (int k = me + 1; k < nn; ++k) {
            const int c = accept_timed(g_net.listen_fd);
            Hello hk{};
            if (c < 0 || xfer(c, nullptr, 0, (char *)&hk, sizeof(hk)) || hk.magic != kMagic || hk.node <= me ||
                hk.node >= nn || g_net.fd[hk.node] >= 0) {
                MV2_ERR("leader of node %d: bad or missing mesh connection", me);
                if (c >= 0) close(c);
                return E_OTHER;
            }
            g_net.fd[hk.node] = c;
        }
    }
    g_net.up = true;
    MV2_DEBUG("inter-node mesh up: node %d of %d", me, nn);
    return net_barrier();
}

// dissemination barrier over the leaders (log2(nnodes) rounds of one-byte tokens)
int net_barrier() {
    World &w = world();
    const int nn = w.nnodes, me = w.node;
    if (nn <= 1) return 0;
    for (int d = 1; d < nn; d <<= 1) {
        const int to = (me + d) % nn, from = (me - d + nn) % nn;
        char t = 1, r = 0;
        int rc = net_send(to, &t, 1);  // one byte never blocks in the socket buffer
        if (!rc) rc = net_recv(from, &r, 1);
        if (rc) {
            MV2_ERR("leaders' barrier (node %d of %d): step %d (token to node %d, from node %d) failed", me, nn, d,
                    to, from);
            return rc;
        }
    }
    return 0;
}

int mesh_setup() {
    World &w = world();
    const int L = w.size, K = w.nnodes, n = w.gsize;
    if (K <= 1 || n > kMeshMaxRanks) return 0;  // no rank mesh: point-to-point stays within nodes
    int port = 0;
    g_mesh.listen_fd = open_listener(nullptr, 0, &port);
    int rc = g_mesh.listen_fd < 0 ? E_OTHER : 0;
    if (w.shm) w.shm->r[w.rank].mesh_port = rc ? -1 : port;
    host_barrier();
    std::vector<int32_t> all((size_t)n, -1);
    std::vector<std::string> ip((size_t)K);
    if (w.rank == 0) {
        // every node's listener ports: a ring of per-node sections over the leaders
        for (int l = 0; l < L; ++l) all[(size_t)w.node * L + l] = w.shm ? w.shm->r[l].mesh_port : port;
        const int me = w.node, right = (me + 1) % K, left = (me - 1 + K) % K;
        const size_t sect = (size_t)L * sizeof(int32_t);
        for (int k = 0; k < K - 1 && !rc; ++k) {
            const int so = (me - k + K) % K, ro = (me - k - 1 + K) % K;
            rc = net_shift(right, &all[(size_t)so * L], sect, left, &all[(size_t)ro * L], sect);
        }
        for (int g = 0; g < n && !rc; ++g)
            if (all[g] < 0) rc = E_OTHER;
        if (w.shm) {
            for (int g = 0; g < n; ++g) w.shm->mesh_port[g] = all[g];
            for (int j = 0; j < K; ++j) {
                if (g_net.ip[j].size() >= sizeof(w.shm->node_ip[j])) {  // dotted IPv4 always fits
                    MV2_ERR("rank mesh: node %d's address '%s' does not fit the control segment", j, g_net.ip[j].c_str());
                    rc = E_OTHER;
                }
                snprintf(w.shm->node_ip[j], sizeof(w.shm->node_ip[j]), "%s", g_net.ip[j].c_str());
            }
            w.shm->net_rc.store(rc);
        }
        for (int j = 0; j < K; ++j) ip[j] = g_net.ip[j];
    }
    host_barrier();
    if (w.shm) {
        rc = w.shm->net_rc.load();
        for (int g = 0; g < n; ++g) all[g] = w.shm->mesh_port[g];
        for (int j = 0; j < K; ++j) ip[j] = w.shm->node_ip[j];
    }
    if (rc) {
        MV2_ERR("rank mesh: a node's listener ports could not be exchanged");
        return rc;
    }
    // connect to every rank of a lower node, accept every rank of a higher one
    g_mesh.fd.assign((size_t)n, -1);
    for (int g = 0; g < w.node * L; ++g) {
        const int c = connect_retry(ip[g / L].c_str(), all[g]);
        const MeshHello h{kMagic, w.grank};
        if (c < 0 || xfer(c, (const char *)&h, sizeof(h), nullptr, 0)) {
            MV2_ERR("rank mesh: cannot connect to rank %d (%s:%d)", g, ip[g / L].c_str(), all[g]);
            return E_OTHER;
        }
        g_mesh.fd[g] = c;
    }
    for (int k = (w.node + 1) * L; k < n; ++k) {
        const int c = accept_timed(g_mesh.listen_fd);
        MeshHello h{};
        if (c < 0 || xfer(c, nullptr, 0, (char *)&h, sizeof(h)) || h.magic != kMagic || h.grank < (w.node + 1) * L ||
            h.grank >= n || g_mesh.fd[h.grank] >= 0) {
            MV2_ERR("rank mesh: bad or missing connection from a higher node");
            if (c >= 0) close(c);
            return E_OTHER;
        }
        g_mesh.fd[h.grank] = c;
    }
    MV2_DEBUG("rank mesh up: rank %d linked to %d ranks of other nodes", w.grank, n - L);
    return 0;
}

int mesh_fd(int grank) { return grank >= 0 && grank < (int)g_mesh.fd.size() ? g_mesh.fd[grank] : -1; }

void net_finalize() {
    for (int &fd : g_mesh.fd)
        if (fd >= 0) {
            close(fd);
            fd = -1;
        }
    if (g_mesh.listen_fd >= 0) close(g_mesh.listen_fd);
    g_mesh.listen_fd = -1;
    for (int &fd : g_net.fd)
        if (fd >= 0) {
            close(fd);
            fd = -1;
        }
    if (g_net.listen_fd >= 0) close(g_net.listen_fd);
    g_net.listen_fd = -1;
    g_net.up = false;
}

}  // namespace mv2
