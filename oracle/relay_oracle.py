"""CPU restatement of the p2pnetwork flood relay (ORACLE -- test infrastructure only).

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may import this module,
and only as the checker / CPU baseline.  The product path never imports oracle/.

What it restates (pj8912/python-p2p-network, read-only at /root/reference):
  * fan-out primitive  Node.send_to_nodes(data, exclude=[sender])   p2pnetwork/node.py:106-112
    -> one Node.send_to_node per connection not excluded, message_count_send += 1 before the
       send                                                         node.py:114-120 (:116)
  * neighbour list     Node.all_nodes = nodes_inbound + nodes_outbound   node.py:75-78
  * receive hook       Node.node_message(node, data)                node.py:334-338, called per
                       packet from NodeConnection.run                nodeconnection.py:186-218
  * app dedup          "keep track which messages you have received" README.md:20 -- a peer
                       forwards a message on first receipt only.
Round-synchronous schedule: all sends of round r-1 arrive in round
r; a receiver handles arrivals in ascending sender id, so the recorded sender (parent) of a
first receipt is the lowest-id neighbour whose copy arrived in that round.  Gossip / churn are
the build-defined variants of SURVEY.md A.3 / A.4 (see oracle/philox.py).

Parity status: pinned -- tests/test_oracle_golden.py checks this module bit-exactly against
the fixtures in tests/golden/, which were produced by driving the reference's own Node /
NodeConnection objects (tests/golden/make_golden.py).

Results: hop[v, m] (round of first receipt, -1 = never), parent[v, m] (-1 at the origin or
never), and per-round stats with the same meaning as p2pg_round_stats.
"""
from dataclasses import dataclass, field

import numpy as np

from . import philox


@dataclass
class RelayResult:
    hop: np.ndarray
    parent: np.ndarray
    rounds: list = field(default_factory=list)

    @property
    def total_relays(self):
        return sum(r["relays"] for r in self.rounds)

    def delivered(self):
        return self.hop >= 0


def _round_stats(rnd, new, deg, relays_per_bit, scatter_words=0):
    """new: bool [V, M] first receipts of round rnd."""
    V, M = new.shape
    W = (M + 63) // 64
    pad = np.zeros((V, W * 64), dtype=bool)
    pad[:, :M] = new
    words = pad.reshape(V, W, 64).any(axis=2)
    per_v = new.sum(axis=1).astype(np.int64)
    active = per_v > 0
    return {
        "round": rnd,
        "new_deliveries": int(per_v.sum()),
        "relays": int((per_v * relays_per_bit).sum()),
        "active_vertices": int(active.sum()),
        "active_words": int(words.sum()),
        "wedges": int((words.sum(axis=1) * deg).sum()),
        "deg_active": int(deg[active].sum()),
        "scatter_words": int(scatter_words),
    }


def _check_csr(rowptr, colidx):
    rowptr = np.asarray(rowptr, dtype=np.int64)
    colidx = np.asarray(colidx, dtype=np.int64)
    V = len(rowptr) - 1
    assert rowptr[0] == 0 and rowptr[-1] == len(colidx)
    return rowptr, colidx, V


def _slots(rowptr, colidx, pairs):
    """Slots of both directions of the undirected pairs (each must exist)."""
    out = []
    for a, b in np.asarray(pairs, dtype=np.int64).reshape(-1, 2):
        for x, y in ((a, b), (b, a)):
            row = colidx[rowptr[x]:rowptr[x + 1]]
            k = int(np.searchsorted(row, y))
            assert k < len(row) and row[k] == y, "removed connection does not exist"
            out.append(rowptr[x] + k)
    return np.asarray(out, dtype=np.int64)


def _apply_changes(rowptr, colidx, add, remove):
    """Topology after connecting `add` and disconnecting `remove` (undirected pairs), CSR
    rows ascending -- Node.connect_with_node / disconnect_with_node between rounds."""
    V = len(rowptr) - 1
    rows = np.repeat(np.arange(V, dtype=np.int64), np.diff(rowptr))
    keep = np.ones(len(colidx), dtype=bool)
    keep[_slots(rowptr, colidx, remove)] = False
    a = np.asarray(add, dtype=np.int64).reshape(-1, 2)
    src = np.concatenate([rows[keep], a[:, 0], a[:, 1]])
    dst = np.concatenate([colidx[keep], a[:, 1], a[:, 0]])
    order = np.lexsort((dst, src))
    src, dst = src[order], dst[order]
    nrp = np.zeros(V + 1, dtype=np.int64)
    np.cumsum(np.bincount(src, minlength=V), out=nrp[1:])
    return nrp, dst.astype(np.int64)


def flood(rowptr, colidx, src, churn_threshold=0, churn_seed=0, max_rounds=1 << 20,
          updates=None):
    """Flood relay with message-id dedup (forward to all connections except the sender).

    updates: {r: (add_pairs, remove_pairs)} -- connection changes after round r.  The sends of
    round r travel on the connections they were made on; those on removed connections are
    lost in flight; the sends of round r+1 on use the new connections (include/p2pgpu.h
    p2pg_update_edges)."""
    updates = updates or {}
    rowptr, colidx, V = _check_csr(rowptr, colidx)
    src = np.asarray(src, dtype=np.int64)
    M = len(src)
    deg = np.diff(rowptr)
    rows = np.repeat(np.arange(V), deg)  # receiver of each directed edge slot
    hop = np.full((V, M), -1, dtype=np.int32)
    parent = np.full((V, M), -1, dtype=np.int32)
    seen = np.zeros((V, M), dtype=bool)
    F = np.zeros((V, M), dtype=bool)
    F[src, np.arange(M)] = True
    seen |= F
    hop[F] = 0
    res = RelayResult(hop, parent)
    # round 0: the origin's send_to_nodes reaches all deg(src) connections
    st = _round_stats(0, F, deg, np.zeros(V, dtype=np.int64))
    st["relays"] = int(deg[src].sum())
    res.rounds.append(st)
    maxdeg = int(deg.max()) if V else 0
    rnd = 0
    while F.any() and rnd < max_rounds:
        rnd += 1
        alive = ~philox.churn_dropped(rnd - 1, rows, colidx, churn_threshold, churn_seed)
        upd = updates.get(rnd - 1)
        if upd is not None:
            alive[_slots(rowptr, colidx, upd[1])] = False
        pending = np.zeros((V, M), dtype=bool)
        contrib = F[colidx] & alive[:, None]  # [E, M]: sender colidx[e] -> receiver rows[e]
        arr = np.zeros((V, M), dtype=bool)
        np.logical_or.at(arr, rows, contrib)
        new = arr & ~seen
        pending[:] = new
        # lowest-id sender: scan each row's (ascending) neighbour slots in order
        for j in range(maxdeg):
            has = deg > j
            if not has.any():
                break
            us = np.nonzero(has)[0]
            e = rowptr[us] + j
            hit = contrib[e] & pending[us]
            if hit.any():
                r_i, m_i = np.nonzero(hit)
                parent[us[r_i], m_i] = colidx[e[r_i]]
                pending[us] &= ~hit
        assert not pending.any()
        if upd is not None:  # the receipts of this round relay on the new connections
            rowptr, colidx = _apply_changes(rowptr, colidx, upd[0], upd[1])
            deg = np.diff(rowptr)
            rows = np.repeat(np.arange(V), deg)
            maxdeg = int(deg.max()) if V else 0
        seen |= new
        hop[new] = rnd
        F = new
        res.rounds.append(_round_stats(rnd, new, deg, deg - 1))
    return res


def gossip(rowptr, colidx, src, fanout, gossip_seed, msg_id_base=0, churn_threshold=0,
           churn_seed=0, max_rounds=1 << 20, updates=None):
    """Push-gossip: on first receipt (or origination) in round r, peer v pushes m to
    min(k, deg v) distinct neighbours picked by Philox(round, v, msg) (sender not excluded).
    updates: as for flood()."""
    updates = updates or {}
    rowptr, colidx, V = _check_csr(rowptr, colidx)
    src = np.asarray(src, dtype=np.int64)
    M = len(src)
    k = int(fanout)
    W = (M + 63) // 64
    deg = np.diff(rowptr)
    hop = np.full((V, M), -1, dtype=np.int32)
    parent = np.full((V, M), -1, dtype=np.int32)
    seen = np.zeros((V, M), dtype=bool)
    F = np.zeros((V, M), dtype=bool)
    F[src, np.arange(M)] = True
    seen |= F
    hop[F] = 0
    res = RelayResult(hop, parent)
    fan = np.minimum(deg, k)
    rnd = 0
    pending_stats = _round_stats(0, F, deg, fan)
    while True:
        # pushes made in round rnd by the round-rnd first receipts F
        vs, ms = np.nonzero(F)
        tgt_l, snd_l, msg_l = [], [], []
        if len(vs):
            d = deg[vs]
            small = d <= k
            for v_i, m_i in zip(vs[small], ms[small]):  # send to every neighbour
                nb = colidx[rowptr[v_i]:rowptr[v_i + 1]]
                tgt_l.append(nb)
                snd_l.append(np.full(len(nb), v_i))
                msg_l.append(np.full(len(nb), m_i))
            big = ~small
            if big.any():
                pk = philox.gossip_picks(rnd, vs[big], ms[big] + msg_id_base, d[big], k, gossip_seed)
                tgt_l.append(colidx[rowptr[vs[big]][:, None] + pk].ravel())
                snd_l.append(np.repeat(vs[big], k))
                msg_l.append(np.repeat(ms[big], k))
        if tgt_l:
            tgt = np.concatenate(tgt_l).astype(np.int64)
            snd = np.concatenate(snd_l).astype(np.int64)
            msg = np.concatenate(msg_l).astype(np.int64)
        else:
            tgt = snd = msg = np.zeros(0, dtype=np.int64)
        keep = ~philox.churn_dropped(rnd, snd, tgt, churn_threshold, churn_seed)
        tgt, snd, msg = tgt[keep], snd[keep], msg[keep]
        # scatter words: distinct (sender, target, word) masks actually pushed
        if len(tgt):
            key = (snd * V + tgt) * W + msg // 64
            pending_stats["scatter_words"] = int(len(np.unique(key)))
        res.rounds.append(pending_stats)
        if not len(vs) or rnd >= max_rounds:
            break
        upd = updates.get(rnd)
        if upd is not None:  # pushes on removed connections are lost; new picks, new lists
            r = np.asarray(upd[1], dtype=np.int64).reshape(-1, 2)
            gone = set(map(tuple, r.tolist())) | set(map(tuple, r[:, ::-1].tolist()))
            if len(tgt) and gone:
                keep = np.array([(int(a), int(b)) not in gone for a, b in zip(snd, tgt)], dtype=bool)
                tgt, snd, msg = tgt[keep], snd[keep], msg[keep]
            rowptr, colidx = _apply_changes(rowptr, colidx, upd[0], upd[1])
            deg = np.diff(rowptr)
            fan = np.minimum(deg, k)
        rnd += 1
        arr = np.zeros((V, M), dtype=bool)
        arr[tgt, msg] = True
        new = arr & ~seen
        best = np.full((V, M), np.iinfo(np.int32).max, dtype=np.int64)
        np.minimum.at(best, (tgt, msg), snd)
        parent[new] = best[new]
        seen |= new
        hop[new] = rnd
        F = new
        pending_stats = _round_stats(rnd, new, deg, fan)
    # drop the trailing empty round's duplicate bookkeeping: the last appended stats is the
    # round with no first receipts (quiescence), matching the engine's final step
    return res
