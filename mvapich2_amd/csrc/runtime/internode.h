// internode.h — leader transport between nodes (the inter-node step of
// MVAPICH2's two-level collectives, create_2level_comm.c:1843 leader_comm).  One TCP stream
// per pair of node leaders (local rank 0 of each node); every other rank talks to its node
// only (IPC arenas, runtime/world.cpp).  Host staging; the reductions stay on the GPU.
#pragma once
#include <stddef.h>

namespace mv2 {

int net_init();      // leaders: bootstrap + full mesh (rank 0's leader serves the rendezvous)
void net_finalize();
int net_barrier();   // leaders only
// blocking exchanges with the leader of node `peer` (both sides issue the matching call)
int net_send(int peer, const void *buf, size_t bytes);
int net_recv(int peer, void *buf, size_t bytes);
int net_sendrecv(int peer, const void *sbuf, size_t sbytes, void *rbuf, size_t rbytes);
// one ring step: send to `to` while receiving from `from`, both directions in flight together
int net_shift(int to, const void *sbuf, size_t sbytes, int from, void *rbuf, size_t rbytes);

// Rank mesh (every rank, after the leaders' bootstrap): one TCP stream between every pair of
// ranks on different nodes, for point-to-point across nodes (runtime/p2p.cpp).  The ports travel
// through the node's control segment and the leaders' links.  Jobs above kMeshMaxRanks ranks get
// no mesh.  mesh_fd: the stream to global rank g, or -1.
int mesh_setup();
int mesh_fd(int grank);

}  // namespace mv2
