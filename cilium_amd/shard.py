"""Multi-GPU plumbing for the classification path.

* Tuples are independent units: a stream is partitioned by a flow hash of
  the 5-tuple, so all packets of a flow land on the same GPU (the property
  RSS gives the reference's per-CPU datapath) and shards need no exchange.
* Tables are replicated on every rank (identical update sequences; compare
  `Engine.checksum()` across ranks).
* The only collective is the integer SUM of the counter delta buffer
  (per-policy-entry packets/bytes + {reason, dir} metrics), after which every
  rank folds the same global delta into its totals.  Integer addition is
  order-independent, so the result is bit-exact against one GPU processing
  the whole stream.
"""
from __future__ import annotations

import numpy as np


def flowhash_np(saddr, daddr, sport, dport, proto) -> np.ndarray:
    """Deterministic 32-bit flow hash (murmur3 finalizer over the 5-tuple),
    cgpu_flow_hash.  Direction-sensitive, like skb->hash for the reference's
    RSS spreading.  uint32 arithmetic wraps mod 2^32."""
    with np.errstate(over="ignore"):
        h = np.asarray(saddr).astype(np.uint32) * np.uint32(0x9E3779B1)
        h ^= np.asarray(daddr).astype(np.uint32)
        h *= np.uint32(0x85EBCA77)
        h ^= (np.asarray(sport).astype(np.uint32) << np.uint32(16)) | np.asarray(dport).astype(np.uint32)
        h *= np.uint32(0xC2B2AE3D)
        h ^= np.asarray(proto).astype(np.uint32)
        h ^= h >> np.uint32(16)
        h *= np.uint32(0x85EBCA6B)
        h ^= h >> np.uint32(13)
        h *= np.uint32(0xC2B2AE35)
        h ^= h >> np.uint32(16)
    return h


def assign_shard_sports(t: dict, world: int, rank: int, seed: int) -> np.ndarray:
    """Source ports that put every tuple of `t` on `rank`: the tuple's own
    sport (or a uniform draw when it has none), redrawn for the tuples whose
    flowhash(5-tuple) % world != rank.  Rank r's batch is then exactly its
    flowhash shard of the stream the ranks generate together (config 4: the
    stream sharded by flowhash % N)."""
    rng = np.random.Generator(np.random.PCG64(seed))
    n = len(t["saddr"])
    if "sport" in t:
        sport = np.array(t["sport"], np.uint16)
    else:
        sport = rng.integers(1024, 65536, n).astype(np.uint16)
    if world == 1:
        return sport
    todo = np.arange(n)
    h = flowhash_np(t["saddr"], t["daddr"], sport, t["dport"], t["proto"])
    todo = todo[(h % np.uint32(world)) != rank]
    sport[todo] = rng.integers(1024, 65536, len(todo)).astype(np.uint16)
    while len(todo):
        h = flowhash_np(t["saddr"][todo], t["daddr"][todo], sport[todo], t["dport"][todo],
                        t["proto"][todo])
        todo = todo[(h % np.uint32(world)) != rank]
        sport[todo] = rng.integers(1024, 65536, len(todo)).astype(np.uint16)
    return sport


def _fmix_np(h):
    h = h & np.uint64(0xFFFFFFFF)
    h ^= h >> np.uint64(16)
    h = (h * np.uint64(0x85EBCA6B)) & np.uint64(0xFFFFFFFF)
    h ^= h >> np.uint64(13)
    h = (h * np.uint64(0xC2B2AE35)) & np.uint64(0xFFFFFFFF)
    h ^= h >> np.uint64(16)
    return h


def fold6_np(a16) -> np.ndarray:
    """tables.h fold6: (n, 16) uint8 addresses -> u32 (four LE words mixed)"""
    w = np.ascontiguousarray(a16, np.uint8).view("<u4").reshape(-1, 4).astype(np.uint64)
    h = _fmix_np(w[:, 3] ^ np.uint64(0x6B43A9B5))
    h = _fmix_np(w[:, 2] ^ h)
    h = _fmix_np(w[:, 1] ^ h)
    return _fmix_np(w[:, 0] ^ h).astype(np.uint32)


def flowhash6_np(saddr16, daddr16, sport, dport, proto) -> np.ndarray:
    """cgpu_flow_hash6: flowhash_np over the folded IPv6 addresses"""
    return flowhash_np(fold6_np(saddr16), fold6_np(daddr16), sport, dport, proto)


def shard_of(t: dict, world: int) -> np.ndarray:
    """Owning rank of every tuple: flowhash(5-tuple) % world."""
    sport = t.get("sport", np.zeros_like(t["dport"]))
    return (flowhash_np(t["saddr"], t["daddr"], sport, t["dport"], t["proto"]) %
            np.uint32(world)).astype(np.int64)


def pairhash_np(saddr, daddr) -> np.ndarray:
    """Direction-free 32-bit hash of the unordered address pair.  The
    stateful path (cgpu_classify_v4_ct) shards by it: every
    conntrack key a packet reads or writes (forward, reply and ICMP-related
    tuples) carries that pair, so each rank's conntrack map holds exactly the
    entries of its own packets and the shards never exchange state."""
    a = np.asarray(saddr).astype(np.uint64)
    b = np.asarray(daddr).astype(np.uint64)
    lo, hi = np.minimum(a, b), np.maximum(a, b)
    h = (lo * np.uint64(0x9E3779B1)) & np.uint64(0xFFFFFFFF)
    h ^= hi
    h = (h * np.uint64(0x85EBCA77)) & np.uint64(0xFFFFFFFF)
    h ^= h >> np.uint64(15)
    h = (h * np.uint64(0xC2B2AE3D)) & np.uint64(0xFFFFFFFF)
    h ^= h >> np.uint64(16)
    return h.astype(np.uint32)


def pairhash6_np(saddr16, daddr16) -> np.ndarray:
    """pairhash_np over the folded IPv6 addresses (tables.h fold6)."""
    return pairhash_np(fold6_np(saddr16), fold6_np(daddr16))


def ct_shard_of(t: dict, world: int) -> np.ndarray:
    """Owning rank of every packet of the stateful path: pairhash % world.

    Capacity: every rank's conntrack map is a whole CT_MAP_SIZE (cfg.ct_max),
    as every node's cilium_ct4_global is in the reference, so the ranks
    together hold up to world x ct_max entries.  The union of the rank maps
    equals the one-process map while no map reaches ct_max; past that the
    DROP_CT_CREATE_FAILED set depends on which shard fills first (and, within
    one map, on lane order: cgpu.h), so parity is defined below capacity
    only.  A deployment that wants the aggregate of one map passes
    ct_max // world per rank."""
    if np.asarray(t["saddr"]).ndim == 2:
        return (pairhash6_np(t["saddr"], t["daddr"]) % np.uint32(world)).astype(np.int64)
    return (pairhash_np(t["saddr"], t["daddr"]) % np.uint32(world)).astype(np.int64)


def conn_shard_of(t: dict, world: int) -> np.ndarray:
    """RSS-style owner of every packet of the service path: a hash of the
    local side of its connection (the endpoint address and port, the
    protocol), the same for both directions whatever address the remote side
    shows (service VIP or backend).  Used to thread the CPU restatement of
    cgpu_classify_v{4,6}_ctlb (bench.py cpu_baseline); unlike ct_shard_of
    it is not a partition into independent conntrack groups (ICMP-related and
    address entries cross connections), so bench.py compares its result with
    the sequential run."""
    eg = (np.asarray(t["flags"]) & 1).astype(bool)
    sa, da = np.asarray(t["saddr"]), np.asarray(t["daddr"])
    if sa.ndim == 2:
        sa, da = fold6_np(sa), fold6_np(da)
    loc = np.where(eg, sa, da).astype(np.uint32)
    lport = np.where(eg, t["sport"], t["dport"]).astype(np.uint32)
    return (flowhash_np(loc, np.zeros_like(loc), lport, np.zeros_like(lport), t["proto"]) %
            np.uint32(world)).astype(np.int64)


def _addr_ids(a) -> np.ndarray:
    a = np.asarray(a)
    return (fold6_np(a) if a.ndim == 2 else a).astype(np.uint64)


def _pairkey(a, b) -> np.ndarray:
    lo, hi = np.minimum(a, b), np.maximum(a, b)
    return (lo << np.uint64(32)) | hi


def svc_component_shard_of(t: dict, svc_keys, svc_vals, world: int, loopback: int = 0) -> np.ndarray:
    """An EXACT partition of the service path (cgpu_classify_v{4,6}_ctlb) into
    independent conntrack groups, for threading its CPU restatement and for
    sharding it across GPUs.  ct_shard_of is not one: a service packet's
    keys live in its own address pair {client, VIP} (the CT_SERVICE entry,
    lb.h:700-775), in the pair of the backend it is translated to {client,
    backend} (the conntrack entries, conntrack.h:649-744) and, through
    ct_create4's address entry, in {backend, backend} or, on loopback, in
    {IPV4_LOOPBACK, client} / {backend, 0}.  Every packet is a node's member
    (its own pair); a packet that may be a service packet (egress to an
    address the service map holds) links its pair with every pair it could
    reach through ANY backend of that address (the selection itself depends
    on state, so all of them), and the connected components of those links
    are closed under every key any of their packets touches: each component
    runs alone and the union of the runs is the sequential result.  IPv6
    addresses enter as their 32-bit folds (a collision only merges
    components).  Returns a shard id per packet: component hash % world."""
    from scipy.sparse import coo_matrix
    from scipy.sparse.csgraph import connected_components
    sa, da = _addr_ids(t["saddr"]), _addr_ids(t["daddr"])
    node = _pairkey(sa, da)
    k = np.asarray(svc_keys)
    v = np.asarray(svc_vals)
    vip = _addr_ids(k["address"])
    back = k["slave"] != 0
    bvip, btgt = vip[back], _addr_ids(v["target"][back])
    order = np.argsort(bvip, kind="stable")
    bvip, btgt = bvip[order], btgt[order]
    uvip, first, cnt = np.unique(bvip, return_index=True, return_counts=True)
    eg = (np.asarray(t["flags"]) & 1).astype(bool)
    cand = eg & np.isin(da, np.unique(vip))
    # distinct (client, address) pairs of the candidates, each with every
    # backend row of that address
    cv = np.unique(np.stack([sa[cand], da[cand]], 1), axis=0) if cand.any() else np.zeros((0, 2), np.uint64)
    vi = np.searchsorted(uvip, cv[:, 1])
    has = (vi < len(uvip))
    has[has] &= uvip[vi[has]] == cv[has, 1]
    cv, vi = cv[has], vi[has]
    rep = cnt[vi]
    c_rep = np.repeat(cv[:, 0], rep)
    v_rep = np.repeat(cv[:, 1], rep)
    off = np.arange(rep.sum()) - np.repeat(np.cumsum(rep) - rep, rep)
    b_rep = btgt[np.repeat(first[vi], rep) + off]
    src = _pairkey(c_rep, v_rep)
    lb = np.uint64(loopback)
    loop = b_rep == c_rep
    ends = [(src, _pairkey(c_rep, b_rep)), (_pairkey(c_rep, b_rep), _pairkey(b_rep, b_rep)),
            (src[loop], _pairkey(np.full(int(loop.sum()), lb, np.uint64), c_rep[loop])),
            (src[loop], _pairkey(b_rep[loop], np.zeros(int(loop.sum()), np.uint64)))]
    keys = np.concatenate([node] + [x for e in ends for x in e])
    uk, inv = np.unique(keys, return_inverse=True)
    n = len(node)
    ei, pos = [], n
    for a_, b_ in ends:
        m = len(a_)
        ei.append((inv[pos:pos + m], inv[pos + m:pos + 2 * m]))
        pos += 2 * m
    r = np.concatenate([x for x, _ in ei]) if ei else np.zeros(0, np.int64)
    c = np.concatenate([y for _, y in ei]) if ei else np.zeros(0, np.int64)
    g = coo_matrix((np.ones(len(r), np.int8), (r, c)), shape=(len(uk), len(uk)))
    _, lab = connected_components(g, directed=False)
    comp = lab[inv[:n]].astype(np.uint64)
    return (_fmix_np(comp ^ np.uint64(0x5BD1E995)) % np.uint64(world)).astype(np.int64)


def take(t: dict, idx) -> dict:
    return {k: np.ascontiguousarray(v[idx]) for k, v in t.items()}


def init_counter_comm(engine, rank: int, world: int, group=None) -> None:
    """Join the engine's counter communicator (cgpu_comm_id_create /
    cgpu_comm_init, RCCL linked into libcgpu.so): rank 0 creates the id and
    hands it to the other ranks over `group` -- the out-of-band channel the
    agent would use.  Collective: returns once every rank joined."""
    import torch.distributed as dist
    box = [engine.comm_id() if rank == 0 else None]
    dist.broadcast_object_list(box, src=0, group=group)
    engine.comm_init(box[0], world, rank)


def reduce_counters(engine, world: int, stream=None) -> None:
    """The per-step counter reduction of the sharded stream: the RCCL u64
    SUM of every rank's delta buffer (cgpu_counters_allreduce), after which
    each rank's cgpu_counter_fold adds the same global delta to its totals.
    Nothing to do for one rank."""
    if world > 1:
        engine.counters_allreduce(stream)


def allreduce_counters(delta, group=None):
    """The same SUM over torch tensors, for the CPU restatement's counters in
    the gloo tests (tests/test_multi_gloo.py): u64 counters travel as their
    int64 bit pattern (two's-complement addition is the same mod 2^64)."""
    import torch.distributed as dist
    dist.all_reduce(delta, op=dist.ReduceOp.SUM, group=group)
    return delta
