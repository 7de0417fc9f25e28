"""Rank-by-rank restatements of the MVAPICH2 2.3.7 algorithms for a user
MPI_Op (TEST INFRASTRUCTURE: the expected results of the user-op GPU tests).

fn(inp, io) returns the new inout, i.e. the user function's
`inoutvec = invec op inoutvec`; every call below is one uop(in, inout) of the
cited reference code.  The algorithm is the one the reference selects
(oracle.allreduce_select / reduce_select / reduce_scatter_select with the
user-op kind)."""
import numpy as np

from oracle import oracle


def pof2_of(n):
    p = 1
    while p * 2 <= n:
        p *= 2
    return p


def linear(xs, fn):
    """reduce_shmem (allreduce_osu.c:1569-1583): x0 inout, uop(x_i, acc)"""
    acc = xs[0].copy()
    for x in xs[1:]:
        acc = fn(x, acc)
    return acc


def tree(xs, fn, deg=4):
    """mv2_shm_tree_reduce (ch3_shmem_coll.c:4272-4359) at local rank 0"""
    n = len(xs)
    slot = [x.copy() for x in xs]
    for g in range(0, n, deg):
        for i in range(g + 1, min(g + deg, n)):
            slot[g] = fn(slot[i], slot[g])
    for g in range(deg, n, deg):
        slot[0] = fn(slot[g], slot[0])
    return slot[0]


def rd(xs, fn, commute):
    """pt2pt_rd / pt2pt_rs recursive doubling (allreduce_osu.c:455-600, :802-851): per-rank results"""
    n = len(xs)
    pof2 = pof2_of(n)
    rem = n - pof2
    rb = [x.copy() for x in xs]
    newrank, real = [0] * n, [0] * pof2
    for r in range(n):
        if r < 2 * rem:
            if r % 2 == 0:
                newrank[r] = -1
            else:
                rb[r] = fn(xs[r - 1], rb[r])
                newrank[r] = r // 2
        else:
            newrank[r] = r - rem
        if newrank[r] >= 0:
            real[newrank[r]] = r
    mask = 1
    while mask < pof2:
        prev = [rb[real[nr]].copy() for nr in range(pof2)]
        for nr in range(pof2):
            r, dst = real[nr], real[nr ^ mask]
            tmp = prev[nr ^ mask]
            rb[r] = fn(tmp, rb[r]) if (commute or dst < r) else fn(rb[r], tmp)
        mask <<= 1
    for r in range(0, 2 * rem, 2):
        rb[r] = rb[r + 1]
    return rb


def ring_chunks(xs, fn, count):
    """MPIR_Allreduce_pt2pt_ring_MV2 (allreduce_osu.c:3925-3958) over (count/n)*n elements"""
    n = len(xs)
    cc = count // n
    out = []
    for c in range(n):
        blk = slice(c * cc, (c + 1) * cc)
        acc = xs[c][blk].copy()
        for k in range(1, n):
            acc = fn(xs[(c + k) % n][blk], acc)
        out.append(acc)
    return np.concatenate(out) if out else xs[0][:0].copy()


def allreduce(xs, fn, commute, dtype_handle, count, in_place=False, nbytes=None, stride=0, slot=32768):
    """nbytes: the call's count * type size when the elements are of a derived type
    (the selection depends on it; the algorithms on the element count).  stride: count x extent;
    reduce_shmem from the shmem slot on (allreduce_osu.c:1521-1526) runs MPICH's MPIR_Reduce_intra
    to rank 0 — binomial for a user op (reduce.c:874-894) — and broadcasts rank 0's result"""
    n = len(xs)
    if nbytes is None:
        sel = oracle.allreduce_select(n, count, dtype_handle, in_place, 1 if commute else 2)
    else:
        sel = oracle.allreduce_select(n, nbytes, 0x4c00010d, in_place, 1 if commute else 2)  # MPI_BYTE
    algo = oracle.ALGOS[sel]
    if algo == "topo_tree":
        return [tree(xs, fn)] * n
    if algo == "shmem_linear":
        if stride >= slot:
            return [binomial(xs, fn, 0, commute)] * n
        return [linear(xs, fn)] * n
    if algo == "ring_wrapper":
        main = 0 if (in_place or count < n) else (count // n) * n
        rest = rd([x[main:] for x in xs], fn, commute)
        if not main:
            return rest
        ring = ring_chunks(xs, fn, count)
        return [np.concatenate([ring, rest[r]]) for r in range(n)]
    if algo == "pt2pt_rd":
        return rd(xs, fn, commute)
    raise NotImplementedError(algo)


def binomial(xs, fn, root, commute):
    """MPIR_Reduce_binomial_MV2 (reduce_osu.c:577-663)"""
    n = len(xs)
    lroot = root if commute else 0
    rb = [x.copy() for x in xs]
    mask = 1
    while mask < n:
        for rel in range(n):
            if rel & (mask - 1) or rel & mask or (rel | mask) >= n:
                continue
            me, frm = (rel + lroot) % n, ((rel | mask) + lroot) % n
            rb[me] = fn(rb[frm], rb[me]) if commute else fn(rb[me], rb[frm])
        mask <<= 1
    return rb[lroot]


def knomial(xs, fn, root, k):
    """MPIR_Reduce_knomial_MV2 (reduce_osu.c:1569-1835), request-index (all-arrived) order"""
    n = len(xs)

    def node(rank):
        rel = (rank - root) % n
        mask = 1
        while mask < n:
            if rel % (k * mask):
                break
            mask *= k
        mask //= k
        src = []
        m = mask
        while m > 0:
            for j in range(1, k):
                if rel + m * j < n:
                    src.append((rank + m * j) % n)
            m //= k
        acc = xs[rank].copy()
        for c in reversed(src):
            acc = fn(node(c), acc)
        return acc
    return node(root)


def redscat_gather(xs, fn, count, allreduce_pre=False):
    """MPIR_Reduce_redscat_gather_MV2 (reduce_osu.c:718-1100) for a commutative op: the pre-step (odd
    ranks below 2 * rem hand their operand to rank - 1, which computes uop(tmp, recvbuf)), recursive
    halving over pof2 blocks (the last takes the remainder; each step uop(tmp, recvbuf) on the kept
    half), then the gather: the result every rank's blocks make up.  allreduce_pre: the pre-step of
    MPIR_Allreduce_pt2pt_rs_MV2 instead (allreduce_osu.c:852-1000: even ranks hand theirs to rank + 1),
    whose reduce-scatter + allgather is otherwise the same"""
    n = len(xs)
    pof2 = pof2_of(n)
    rem = n - pof2
    rb = [x.copy() for x in xs]
    for r in range(0, 2 * rem, 2):
        if allreduce_pre:
            rb[r + 1] = fn(xs[r], rb[r + 1])
        else:
            rb[r] = fn(xs[r + 1], rb[r])
    real = [2 * nr + int(allreduce_pre) if nr < rem else nr + rem for nr in range(pof2)]
    cnts = [count // pof2] * (pof2 - 1) + [count - (count // pof2) * (pof2 - 1)]
    disps = [sum(cnts[:i]) for i in range(pof2)] + [count]
    send_idx, recv_idx, last_idx, own = [0] * pof2, [0] * pof2, [pof2] * pof2, [0] * pof2
    mask = 1
    while mask < pof2:
        snap = [rb[real[nr]].copy() for nr in range(pof2)]
        for nr in range(pof2):
            nd = nr ^ mask
            if nr < nd:
                send_idx[nr] = recv_idx[nr] + pof2 // (mask * 2)
                lo, hi = recv_idx[nr], send_idx[nr]
            else:
                recv_idx[nr] = send_idx[nr] + pof2 // (mask * 2)
                lo, hi = recv_idx[nr], last_idx[nr]
            a, b = disps[lo], disps[hi]
            if b > a:
                rb[real[nr]][a:b] = fn(snap[nd][a:b], snap[nr][a:b])
            own[nr] = lo
            send_idx[nr] = recv_idx[nr]
        mask <<= 1
        if mask < pof2:
            for nr in range(pof2):
                last_idx[nr] = recv_idx[nr] + pof2 // mask
    out = xs[0].copy() if pof2 == 1 else np.empty_like(xs[0])
    if pof2 > 1:
        for nr in range(pof2):
            i = own[nr]
            out[disps[i]:disps[i + 1]] = rb[real[nr]][disps[i]:disps[i + 1]]
    else:
        out = rb[0]
    return out


def reduce(xs, fn, commute, dtype_handle, count, root):
    n = len(xs)
    a, kf, root0 = oracle.reduce_select(n, count, dtype_handle, 1 if commute else 2)
    algo = oracle.ALGOS[a]
    if algo == "shmem_linear":
        return linear(xs, fn)
    if algo == "binomial":
        return binomial(xs, fn, root, commute)
    if algo == "knomial":
        return knomial(xs, fn, 0 if root0 else root, kf)
    if algo == "reduce_topo":
        return tree(xs, fn, kf)
    raise NotImplementedError(algo)


def reduce_scatter(xs, fn, dtype_handle, counts, algo=None):
    """commutative user op: MPIR_Reduce_scatter_MV2's choice (red_scat_osu.c:1859-1896; the
    one-node table entry unless `algo` names it); every block"""
    n = len(xs)
    disps = np.concatenate([[0], np.cumsum(counts)]).astype(int)
    algo = algo or oracle.ALGOS[oracle.reduce_scatter_select(counts, dtype_handle)]
    blk = lambda x, b: x[disps[b]:disps[b + 1]]
    out = []
    if algo == "rs_ring":      # red_scat_osu.c:1290-1336
        for b in range(n):
            acc = blk(xs[(b + 1) % n], b).copy()
            for k in range(2, n + 1):
                acc = fn(acc, blk(xs[(b + k) % n], b))
            out.append(acc)
    elif algo == "rs_pairwise":  # :867-989
        for r in range(n):
            acc = blk(xs[r], r).copy()
            for i in range(1, n):
                acc = fn(blk(xs[(r - i) % n], r), acc)
            out.append(acc)
    elif algo == "rs_basic":   # :300-422: MPIR_Reduce_MV2(total, root 0) + scatter
        full = reduce(xs, fn, True, dtype_handle, int(disps[-1]), 0)
        out = [blk(full, b) for b in range(n)]
    elif algo == "rs_rec_halving":  # :537-760
        pof2 = pof2_of(n)
        rem = n - pof2
        res = [x.copy() for x in xs]
        newrank, real = [0] * n, [0] * pof2
        for r in range(n):
            if r < 2 * rem:
                if r % 2 == 0:
                    newrank[r] = -1
                else:
                    res[r] = fn(res[r - 1], res[r])
                    newrank[r] = r // 2
            else:
                newrank[r] = r - rem
            if newrank[r] >= 0:
                real[newrank[r]] = r
        newcnts = []
        for i in range(pof2):
            old = i * 2 + 1 if i < rem else i + rem
            newcnts.append(counts[old] + counts[old - 1] if old < 2 * rem else counts[old])
        nd = np.concatenate([[0], np.cumsum(newcnts)]).astype(int)
        send_idx, recv_idx, last_idx = [0] * pof2, [0] * pof2, [pof2] * pof2
        mask = pof2 >> 1
        while mask > 0:
            lo, hi = [0] * pof2, [0] * pof2
            for nr in range(pof2):
                if nr < nr ^ mask:
                    send_idx[nr] = recv_idx[nr] + mask
                    lo[nr], hi[nr] = recv_idx[nr], send_idx[nr]
                else:
                    recv_idx[nr] = send_idx[nr] + mask
                    lo[nr], hi[nr] = recv_idx[nr], last_idx[nr]
            prev = [r.copy() for r in res]
            for nr in range(pof2):
                r, d = real[nr], real[nr ^ mask]
                a, b = nd[lo[nr]], nd[hi[nr]]
                if b > a:
                    res[r][a:b] = fn(prev[d][a:b], prev[r][a:b])
                send_idx[nr] = recv_idx[nr]
                last_idx[nr] = recv_idx[nr] + mask
            mask >>= 1
        for r in range(n):
            holder = r + 1 if (r < 2 * rem and r % 2 == 0) else r
            out.append(blk(res[holder], r))
    else:
        raise NotImplementedError(algo)
    return out


def _mirror(x, bits):
    """mirror_permutation (red_scat_osu.c:90-103): the low `bits` bits reversed"""
    r = x & ~((1 << bits) - 1)
    for i in range(bits):
        r |= ((x >> i) & 1) << (bits - 1 - i)
    return r


def reduce_scatter_noncomm(xs, fn, counts):
    """MPIR_Reduce_scatter_non_comm_MV2 (red_scat_osu.c:1367-1760) for a non-commutative op: every
    rank's block, rank by rank.  Power-of-two size with equal counts: MPIR_Reduce_scatter_noncomm_MV2
    (:132-290), the blocks mirror-permuted then halved; else recursive doubling over the whole
    buffer with the non-power-of-two hand-off inside subtrees (:1478-1722)."""
    n = len(xs)
    pof2, lg = 1, 0
    while pof2 < n:
        pof2 <<= 1
        lg += 1
    disps = [sum(counts[:r]) for r in range(n)]
    total = sum(counts)
    if pof2 == n and len(set(counts)) == 1:
        bs = counts[0]
        buf = []  # per rank: the mirror-permuted blocks, then the double buffer's current inout
        for r in range(n):
            b = np.empty_like(xs[r][:total])
            for i in range(n):
                m = _mirror(i, lg)
                b[m * bs:(m + 1) * bs] = xs[r][i * bs:(i + 1) * bs]
            buf.append(b)
        send_off, recv_off, size = [0] * n, [0] * n, total
        for k in range(lg):
            size //= 2
            snap = [b.copy() for b in buf]
            for r in range(n):
                peer = r ^ (1 << k)
                if r > peer:
                    recv_off[r] += size
                else:
                    send_off[r] += size
            for r in range(n):
                peer = r ^ (1 << k)
                ro = recv_off[r]
                incoming = snap[peer][ro:ro + size]  # the peer sent its send range = my recv range
                mine = snap[r][ro:ro + size]
                # rank > peer: op(received, mine) into mine; else op(mine, received) into received
                buf[r][ro:ro + size] = fn(incoming, mine) if r > peer else fn(mine, incoming)
                send_off[r] = recv_off[r]
        return [buf[r][recv_off[r]:recv_off[r] + counts[r]].copy() for r in range(n)]
    # recursive doubling
    res = [x[:total].copy() for x in xs]
    rcv = [np.empty_like(x[:total]) for x in xs]

    def blocks_outside(root, mask):
        lo, hi = disps[root] if root < n else total, disps[root + mask] if root + mask < n else total
        return [(0, lo), (hi, total)]

    mask, i = 1, 0
    while mask < n:
        got = [False] * n
        dtr = [((r ^ mask) >> i) << i for r in range(n)]
        mtr = [(r >> i) << i for r in range(n)]
        snap = [x.copy() for x in res]
        for r in range(n):
            dst = r ^ mask
            if dst < n:  # MPIC_Sendrecv: the blocks outside dst's subtree, from dst's results
                for a, b in blocks_outside(dtr[r], mask):
                    rcv[r][a:b] = snap[dst][a:b]
                got[r] = True
        # non-power-of-two: ranks with data hand their received blocks to the subtree's others
        k = mask.bit_length() - 1
        tm = mask >> 1
        while tm:
            moves = []
            for r in range(n):
                if dtr[r] + mask <= n:
                    continue
                npc = n - mtr[r] - mask
                d = r ^ tm
                root = (r >> k) << k
                if d > r and r < root + npc and root + npc <= d < n:
                    moves.append((r, d))
            for s, d in moves:
                for a, b in blocks_outside(dtr[d], mask):
                    rcv[d][a:b] = rcv[s][a:b]
                got[d] = True
            tm >>= 1
            k -= 1
        for r in range(n):
            if not got[r]:
                continue
            for a, b in blocks_outside(dtr[r], mask):
                if b <= a:
                    continue
                if dtr[r] < mtr[r]:
                    res[r][a:b] = fn(rcv[r][a:b], res[r][a:b])
                else:
                    res[r][a:b] = fn(res[r][a:b], rcv[r][a:b])
        mask <<= 1
        i += 1
    return [res[r][disps[r]:disps[r] + counts[r]].copy() for r in range(n)]
