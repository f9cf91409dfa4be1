"""Headline benchmark: Mpps of verdict-exact L3/L4 classification (ipcache
LPM identity + per-endpoint policy-map cascade) per BASELINE.json, and the
fraction of the HBM roofline.

    python bench.py [--gpus N --steps K --warmup W]
    python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N

A step = one classify pass over one 64M-tuple batch already resident in HBM
(config 2: 100k IPv4 ipcache prefixes + 64k policy entries), plus the RCCL
all-reduce of the per-entry/per-reason counter deltas (N > 1: the product's
cgpu_counters_allreduce, shard.reduce_counters) and their fold into the
totals.  Tables are replicated (same seed on every rank).  At N > 1 (config
4) rank r's batch is its flowhash(5-tuple) % N shard of the stream the ranks
generate together: per-rank seeded tuples whose source port is drawn so the
tuple hashes to r (shard.assign_shard_sports, asserted), so per-GPU work is
fixed (weak scaling) and the stream is N x 64M tuples per step.
Rank 0 prints one JSON line.

Other BASELINE configs (not the headline line; run them explicitly):
  --config cascade   config 5 whole, "prefilter -> ipcache -> policy -> LB":
                     the netdev's XDP prefilter (bpf_xdp.c check_v4: 16k dyn4
                     prefixes + 200k fix4 /32s, then the local-endpoint check)
                     in front of every ingress tuple and the egress service
                     step over 1M services (bpf_lxc.c:444-469) in front of
                     every egress tuple, both fused into the classify kernel
                     (cgpu_classify_v4_cascade)
  --config pf6       config 3: XDP IPv6 prefilter over 1M deny prefixes
  --config frames    config 2 tables, the batch as raw Ethernet frames in
                     64-byte ring slots (cgpu_classify_frames: header parse
                     of bpf_lxc.c / conntrack.h fused with the classify)
  --config ct        config 2 tables + stateful conntrack:
                     cgpu_classify_v4_ct over 64M packets of 2M connections,
                     the cilium_ct4_global map emptied at the start of every
                     step (cgpu_ct4_flush, timed), so each step creates,
                     updates and reply-skips the same way; parity on the
                     whole batch and the CPU baseline from the restatement
                     threaded over address-pair shards (pairs are independent
                     conntrack groups, so the threaded run is exact)
  --config ctlb      config 2 tables + 1M services + conntrack behind the
                     STATEFUL service step (cgpu_classify_v4_ctlb: lb4_local
                     with CONNTRACK, CT_SERVICE entries, stored slaves,
                     ct_create4's address entries): 64M packets of 2M
                     connections (40 % to services), map emptied each step,
                     the translated daddr / dport written; parity against the
                     sequential restatement over the whole batch, the CPU
                     baseline threaded by connection
  --config ctlb6     ctlb over IPv6 (cgpu_classify_v6_ctlb, 100k IPv6 services)
  --config ct6       ct over IPv6 (cilium_ct6_global, cgpu_classify_v6_ct):
                     100k IPv6 ipcache prefixes + 64k policy keys, 64M packets
                     of 2M connections, parity on the whole batch
  --config mapstate  L3 MapState compilation: the label
                     decision of computeDesiredL3PolicyMapEntries for 100
                     endpoints x 65536 identities over a 1000-rule repository
                     (cgpu_l3_compile, host tables in, allow matrix out)
  --config cpu       config 1 sizes
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "Mpps classified (LPM ipcache + policy map) at 1/2/4/8 GPUs; % HBM roofline"
HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md: HBM3E 8.0 TB/s spec
B_IN, B_OUT = 18, 8    # v4 classify tuple bytes in / out
B_IN_PF6, B_OUT_PF6 = 33, 1  # v6 prefilter
B_IN_V6 = 42           # v6 classify: saddr 16 + daddr 16 + dport proto flags len ep
FRAME_STRIDE = 64      # --config frames: ring slot bytes (Ethernet + IPv4 + TCP fit)
B_IN_FRAMES = FRAME_STRIDE + 4 + 1 + 2  # slot + len + flags + ep
B_IN_CT, B_OUT_CT = 22, 9  # saddr daddr sport dport proto l4(2) flags len ep / verdict identity ct_ret
B_IN_CT6 = 46              # the same with 16-byte addresses
CT_PKTS_PER_CONN = 32


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def host_cpu():
    """The timing host: CPU model, nproc, usable CPUs (affinity) and the
    cgroup CPU quota, for cpu_baseline.sample."""
    model = "unknown"
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                model = line.split(":", 1)[1].strip()
                break
    except OSError:
        pass
    quota = "none"
    try:
        q, per = open("/sys/fs/cgroup/cpu.max").read().split()
        quota = "none" if q == "max" else f"{int(q) / int(per):.1f} CPUs"
    except (OSError, ValueError):
        pass
    aff = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else os.cpu_count()
    return f"{model}; nproc {os.cpu_count()}, affinity {aff}, cgroup quota {quota}"


WORKLOADS = {
    "gpu": "config2: 100k IPv4 ipcache LPM + 64k policy entries (4 ep x 16k), "
           "64M-tuple batches per GPU, bit-exact verdicts",
    "cpu": "config1 (CPU-scale)",
    "v6": "IPv6 classify at config-2 size: 100k IPv6 ipcache prefixes (1024 /48 sites under 64 "
          "/16 roots; /128 40%, /64 30%, /56 10%, /48 7%, /96 5%, /112 5%, /32 3%) + 64k policy "
          "entries (4 ep x 16k), 64M-tuple batches per GPU, bit-exact verdicts",
    "cascade": "config5: XDP prefilter on ingress (bpf_xdp.c check_v4: 16k dyn4 LPM prefixes + 200k fix4 "
               "/32s on saddr, then daddr in the 4 local endpoints; ~5% of ingress tuples from the deny "
               "set, 1% to no endpoint) | 1M IPv4 services on egress (lb4_local, backends ~Geom(0.3) cap "
               "16, 30% of egress tuples to a service) -> ipcache(post-DNAT) -> policy over config-2 "
               "tables, 64M-tuple batches per GPU, bit-exact verdicts",
    "pf6": "config3: XDP IPv6 prefilter, 1M deny prefixes (/32..../128, /128 in fix) under 256 "
           "/24 roots + 4k endpoints, 64M packets per GPU",
    "frames": "config2 tables, 64M raw Ethernet/IPv4/TCP|UDP frames per GPU in 64-byte slots: "
              "header parse (revalidate, ihl, frag, ct_lookup4 ports) fused with ipcache + policy, "
              "bit-exact verdicts",
    "mapstate": "L3 MapState compilation: 1000 rules (selectors over 3 label sources, In/NotIn/"
                "Exists/DoesNotExist, FromRequires, L4-restricted blocks) x 100 endpoints x 65536 "
                "identities, both directions, bit-exact vs the restatement",
    "ct": "config2 tables + stateful conntrack (cilium_ct4_global, SURVEY §8f row 3): 64M packets "
          "per GPU of 2M TCP/UDP/ICMP connections (~32 packets each, both directions, ICMP errors), "
          "map emptied each step: ct_lookup4 -> ipcache -> policy -> reply/related skip, "
          "ct_create4 / delete, bit-exact",
    "ctlb": "config2 tables + 1M IPv4 services + stateful conntrack behind the stateful service step "
            "(cgpu_classify_v4_ctlb, lb4_local with CONNTRACK): 64M packets per GPU of 2M "
            "connections (~32 packets each, 40 % to services, 0.01 % loopback backends), map emptied "
            "each step: CT_SERVICE lookup/create + slave reuse -> ct_lookup4 -> ipcache -> policy -> "
            "ct_create4 with the service's state and address entry, bit-exact",
    "ctlb6": "IPv6 tables at config-2 size + 100k IPv6 services + stateful conntrack behind the IPv6 "
             "stateful service step (cgpu_classify_v6_ctlb, lb6_local with CONNTRACK over "
             "cilium_ct6_global): 64M packets per GPU of 2M connections (~32 packets each, 40 % to "
             "services), map emptied each step: CT_SERVICE lookup/create + slave reuse -> lb6_xlate -> "
             "ct_lookup6 -> ipcache6 -> policy -> ct_create6 with the service's state, bit-exact",
    "ct6": "IPv6 tables at config-2 size (100k IPv6 ipcache prefixes + 64k policy entries) + stateful "
           "conntrack (cilium_ct6_global): 64M packets per GPU of 2M TCP/UDP/ICMPv6 connections, map "
           "emptied each step: ct_lookup6 -> ipcache6 -> policy -> reply/related skip, ct_create6 / "
           "delete, bit-exact",
}


def link_rates(torch, dev, nbytes=1 << 30):
    """Host <-> device copy rates over page-locked memory (GB/s), best of 3:
    each direction alone, and "both": the two directions at once (equal
    bytes on two streams, total bytes over the time) -- the link the
    host-resident line rides on moves columns up and results down together."""
    h = torch.empty(nbytes, dtype=torch.uint8).pin_memory()
    g = torch.empty(nbytes, dtype=torch.uint8, device=dev)
    out = {}
    for name, dst, src in (("h2d", g, h), ("d2h", h, g)):
        best = 0.0
        for _ in range(3):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            dst.copy_(src, non_blocking=True)
            torch.cuda.synchronize()
            best = max(best, nbytes / (time.perf_counter() - t0) / 1e9)
        out[name] = round(best, 2)
    h2 = torch.empty(nbytes, dtype=torch.uint8).pin_memory()
    g2 = torch.empty(nbytes, dtype=torch.uint8, device=dev)
    s_up, s_down = torch.cuda.Stream(dev), torch.cuda.Stream(dev)
    best = 0.0
    for _ in range(3):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        with torch.cuda.stream(s_up):
            g.copy_(h, non_blocking=True)
        with torch.cuda.stream(s_down):
            h2.copy_(g2, non_blocking=True)
        torch.cuda.synchronize()
        best = max(best, 2 * nbytes / (time.perf_counter() - t0) / 1e9)
    out["both"] = round(best, 2)
    del h, g, h2, g2
    return out


def numa_nodes(t, samples=64):
    """NUMA node of a host tensor's pages (move_pages(2) query, sampled):
    where the host-resident line's buffers landed relative to the GPU."""
    import ctypes
    from collections import Counter
    try:
        libc = ctypes.CDLL(None, use_errno=True)
        base, nbytes = t.data_ptr(), t.numel() * t.element_size()
        step = max(4096, (nbytes // samples) & ~4095)
        pages = (ctypes.c_void_p * samples)(*[(base + i * step) & ~4095 for i in range(samples)])
        status = (ctypes.c_int * samples)()
        if libc.syscall(279, 0, samples, pages, None, status, 0) != 0:  # SYS_move_pages
            return None
        return dict(Counter(int(x) for x in status))
    except (OSError, AttributeError):
        return None


def gpu_numa_node(torch, dev):
    try:
        p = torch.cuda.get_device_properties(dev)
        bdf = "%04x:%02x:%02x.0" % (p.pci_domain_id, p.pci_bus_id, p.pci_device_id)
        return int(open(f"/sys/bus/pci/devices/{bdf}/numa_node").read())
    except (OSError, ValueError, AttributeError):
        return None


def pmc_traffic(args):
    """roofline.traffic: the HBM-side bytes per step from a PMC profile of
    the kernels this process actually ran.  profiles/traffic_<config>.json
    (written by tools/pmc_summary.py, copied in from a profile run) carries
    the identity of the library it measured; a profile of another build
    (other sources) is stale and reported as null."""
    from cilium_amd.build import lib_identity
    if getattr(args, "host_tuples", False):
        return None, "not profiled: the host-resident line is bound by the host link", None
    if getattr(args, "ct_persist", 0):
        return None, ("not profiled: profiles/traffic_<config>.json measures the empty-map workload, "
                      "not the steady state"), None
    tj = args.traffic_json or os.path.join(ROOT, "profiles", f"traffic_{args.config}.json")
    if not os.path.exists(tj):
        return None, f"no PMC profile ({os.path.relpath(tj, ROOT)} absent)", None
    try:
        t = json.load(open(tj))
    except (OSError, ValueError):
        return None, f"unreadable {os.path.relpath(tj, ROOT)}", None
    have = lib_identity()
    was = t.get("library") or {}
    same = ((was.get("lib_sha256") and was.get("lib_sha256") == have["lib_sha256"]) or
            (was.get("src_sha256") and was.get("src_sha256") == have.get("src_sha256")))
    if not same or t.get("config") != args.config:
        return None, (f"stale: {os.path.relpath(tj, ROOT)} measured sources "
                      f"{str(was.get('src_sha256'))[:12]} (config {t.get('config')}), this library's "
                      f"sources {str(have.get('src_sha256'))[:12]}"), None
    return (t.get("hbm_bytes_per_step"),
            f"{os.path.relpath(tj, ROOT)}: {t.get('source')}; sources {str(was.get('src_sha256'))[:12]}, "
            f"built at {str(was.get('git_head'))[:12]}",
            {"name": t.get("dominant_kernel"), "hbm_bytes_per_launch": t.get("hbm_bytes_per_launch"),
             "memory_side_atomics_per_step": t.get("memory_side_atomics_per_step",
                                                   t.get("memory_side_atomics_dominant")),
             "l2_requests_per_step": t.get("l2_requests_per_step")})


CEILINGS = os.path.join(ROOT, "profiles", "ceilings.json")
# reference map -> the engine table its lookups gather from (cgpu_table_bytes)
MAP_TABLE = {"ipcache": "ipcache", "policy": "policy", "lb": "lb4", "prefilter": "prefilter",
             "endpoint": "endpoint", "ct": "ct4"}


def tier_rate(ceil, nbytes):
    """Measured random-gather ceiling (G/s) of a table of nbytes: the rate of
    the largest measured table no larger than it (rates fall with size, so
    this never understates what the tier can serve)."""
    g = ceil["gather"]
    floor = g[0][0]
    for s_, _ in g:
        if s_ <= nbytes:
            floor = s_
    # the envelope: no table of at least `floor` bytes measured faster
    return max(r for s_, r in g if s_ >= floor)


def roofline(n, kern_ms, b_in, b_out, probes_total, split, tbytes, v6, dom):
    """The roofline a lookup-bound step cannot beat: three time
    floors from measured ceilings (profiles/ceilings.json), the largest
    bounds the step.
      gather  every reference map lookup (counted per map by the restatement)
              at the random-gather ceiling of the tier its table lives in
              (tier by the table's device bytes): the lookups into tables of
              at least theta bytes take at least their count / R(theta), for
              every theta (the measured tier mixes in ceilings.json obey it)
      atomic  the memory-side atomics the step's kernels issued (PMC,
              stamped profile of this library) at the measured atomic rate
      stream  the tuple columns in and out at the measured stream rates
    frac = floor / measured kernel time of the step."""
    if not os.path.exists(CEILINGS):
        return None
    ceil = json.load(open(CEILINGS))
    t_s = kern_ms * 1e-3
    counts = dict(split)
    counts["ct"] = max(0, int(probes_total) - sum(split.values()))
    per_map = {}
    for m, c in counts.items():
        if not c:
            continue
        tab = MAP_TABLE[m]
        if v6 and tab in ("lb4", "ct4"):
            tab = tab[:-1] + "6"
        nb = int(tbytes.get(tab, 0))
        per_map[m] = {"lookups_per_tuple": round(c / n, 4), "table": tab, "table_bytes": nb,
                      "tier_g_per_s": tier_rate(ceil, nb), "_n": c}
    # every gather into a table of at least theta bytes is served no faster
    # than the measured tier of a theta-byte table, whatever else runs beside
    # it: T >= max over theta of (lookups into tables >= theta) / R(theta)
    # (ceilings.json "mix": measured two-tier mixes stay within this)
    t_gather, theta = 0.0, None
    for m, x in per_map.items():
        t = sum(y["_n"] for y in per_map.values() if y["table_bytes"] >= x["table_bytes"]) / (
            x["tier_g_per_s"] * 1e9)
        if t > t_gather:
            t_gather, theta = t, x["table_bytes"]
    for x in per_map.values():
        del x["_n"]
    look = sum(counts.values())
    comp = {"gather": {"achieved": round(look / t_s / 1e9, 2),
                       "peak": round(look / t_gather / 1e9, 2) if t_gather else None,
                       "unit": "G lookups/s", "frac": round(t_gather / t_s, 4),
                       "binding_table_bytes": theta, "maps": per_map}}
    rd, wr = ceil["stream"]["read_gbs"], ceil["stream"]["write_gbs"]
    t_stream = n * (b_in / (rd * 1e9) + b_out / (wr * 1e9))
    comp["stream"] = {"achieved": round(n * (b_in + b_out) / t_s / 1e9, 1),
                      "peak": round(n * (b_in + b_out) / t_stream / 1e9, 1), "unit": "GB/s",
                      "frac": round(t_stream / t_s, 4), "bytes_in_per_tuple": b_in,
                      "bytes_out_per_tuple": b_out, "read_gbs": rd, "write_gbs": wr}
    at = (dom or {}).get("memory_side_atomics_per_step")
    t_atomic = None
    if at is not None and ceil.get("atomic_g_per_s"):
        t_atomic = at / (ceil["atomic_g_per_s"] * 1e9)
        comp["atomic"] = {"achieved": round(at / t_s / 1e9, 3), "peak": ceil["atomic_g_per_s"],
                          "unit": "G atomics/s", "frac": round(t_atomic / t_s, 4),
                          "atomics_per_step": at, "source": "stamped PMC profile (TCC_EA0_ATOMIC)"}
    else:
        comp["atomic"] = None
    floors = {"gather": t_gather, "stream": t_stream, "atomic": t_atomic or 0.0}
    bound = max(floors, key=floors.get)
    c = comp[bound]
    return {"bound": bound, "achieved": c["achieved"], "peak": c["peak"], "unit": c["unit"],
            "frac": c["frac"], "components": comp,
            "ceilings": f"{os.path.relpath(CEILINGS, ROOT)}: {ceil.get('source')}"}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--config", default="gpu", choices=sorted(WORKLOADS))
    ap.add_argument("--tuples", type=int, default=0, help="tuples per GPU per step")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--host-tuples", action="store_true",
                    help="config 2 with the batch in page-locked host memory (cgpu_classify_v4_host): "
                         "the PCIe-inclusive rate, reported beside the link's ingest bound")
    ap.add_argument("--no-parity", action="store_true",
                    help="skip the restatement entirely (profiling passes: tools/profile.sh)")
    ap.add_argument("--hot-slots", type=int, default=0,
                    help="cgpu_config.hot_counter_slots (LDS counter slots; 0 = library default)")
    ap.add_argument("--schedule", type=int, default=0,
                    help="cgpu_config.schedule (CGPU_SCHED_*, A/B timing of the fallback schedules; "
                         "0 = the tuned default)")
    ap.add_argument("--cpu-threads", type=int, default=0)
    ap.add_argument("--ct-persist", type=int, default=0, metavar="K",
                    help="--config ct / ct6 in steady state: the conntrack map is carried across "
                         "steps (no flush), each step 30 s after the last, and cgpu_ct{4,6}_gc "
                         "(ctmap.GC RemoveExpired) runs before every K-th step on the device map; "
                         "parity against the restatement carried the same way")
    ap.add_argument("--no-rebalance", action="store_true",
                    help="keep the class-based counter slots (no cgpu_counters_rebalance after warmup)")
    ap.add_argument("--traffic-json", default="",
                    help="PMC summary (tools/pmc_summary.py traffic.json) to report as roofline.traffic; "
                         "default profiles/traffic_<config>.json.  Printed only when it was measured "
                         "on the library this process loaded")
    args = ap.parse_args()

    rank = int(os.environ.get("RANK", 0))
    world = int(os.environ.get("WORLD_SIZE", 1))
    local = int(os.environ.get("LOCAL_RANK", 0))
    if args.config == "mapstate":
        return bench_mapstate(args, rank, world, local)
    import numpy as np
    import torch
    import torch.distributed as dist

    from cilium_amd import layouts as L, shard, synth
    from cilium_amd.engine import Engine

    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    if world > 1:
        dist.init_process_group("nccl", device_id=dev)

    if args.host_tuples and args.config not in ("gpu", "frames", "cascade", "v6", "pf6"):
        raise SystemExit("--host-tuples measures the stateless paths: --config gpu, frames, cascade, v6, pf6")
    pf6 = args.config == "pf6"
    cascade = args.config == "cascade"
    frames = args.config == "frames"
    ct6 = args.config in ("ct6", "ctlb6")
    ctlb = args.config in ("ctlb", "ctlb6")
    ct = args.config == "ct" or ct6 or ctlb
    v6 = args.config == "v6"
    cfg = synth.CONFIGS["v6" if ct6 else "gpu" if (pf6 or frames or ct) else args.config]
    n = args.tuples or cfg["n_tuples"]
    t0 = time.time()
    S = None
    if pf6:
        P = synth.make_prefilter6(**synth.PF6_CONFIG)
        tup = synth.make_packets6(P, n, gpu_id=rank)
        log(f"[rank {rank}] v6 prefilter sets ({len(P.dyn6)} dyn, {len(P.fix6)} fix, "
            f"{len(P.ep6)} endpoints) + {n} packets in {time.time() - t0:.1f}s")
        e = Engine(device=local, **P.engine_config())
        synth.load_prefilter6(e, P)
    elif ct:
        T = synth.make_tables6(**cfg) if ct6 else synth.make_tables(**cfg)
        # each rank's stream is its conntrack shard (address pairs with
        # pairhash % world == rank): per-rank maps, no shared state
        if ctlb and ct6:
            S = synth.make_services6(T, 100_000)
            tup, _, seclabels, S = synth.make_ctlb6_workload(T, S, n // CT_PKTS_PER_CONN, gpu_id=rank,
                                                             mean_pkts=CT_PKTS_PER_CONN, world=world,
                                                             loop_frac=1e-4)
        elif ctlb:
            S = synth.make_services(T, synth.CONFIGS["cascade"]["n_services"])
            # loopback backends (an endpoint reaching itself through a
            # service) concentrate on the 4 endpoints' own pairs: a few
            tup, _, seclabels, S = synth.make_ctlb_workload(T, S, n // CT_PKTS_PER_CONN, gpu_id=rank,
                                                            mean_pkts=CT_PKTS_PER_CONN, world=world,
                                                            loop_frac=1e-4)
        else:
            mk = synth.make_ct6_workload if ct6 else synth.make_ct_workload
            tup, _, seclabels = mk(T, n // CT_PKTS_PER_CONN, gpu_id=rank, mean_pkts=CT_PKTS_PER_CONN,
                                   world=world)
        n = min(n, len(tup["saddr"]))
        tup = {k: np.ascontiguousarray(v[:n]) for k, v in tup.items()}
        # entries per connection: ~1.9 plain (forward + ICMP), ~3.4 behind the
        # service step (+ CT_SERVICE + address entries); the map stays under
        # half full so no create meets the capacity edge
        ct_max = 1 << max(20, int(np.ceil(np.log2((4.5 if ctlb else 2.5) * n / CT_PKTS_PER_CONN))))
        log(f"[rank {rank}] synthetic tables ({len(T.ipc_keys)} ipcache, {len(T.pol_keys)} policy) "
            f"+ {n} packets of {n // CT_PKTS_PER_CONN} connections in {time.time() - t0:.1f}s, "
            f"ct_max {ct_max}")
        ecfg = T.engine_config()
        if S is not None:
            ecfg["lb_max_entries"] = len(S.keys)
        e = Engine(device=local, **ecfg, ct_max=ct_max)
        synth.load_engine(e, T)
        synth.load_lxc(e, seclabels)
        if S is not None:
            (synth.load_services6 if ct6 else synth.load_services)(e, S)
    elif v6:
        T = synth.make_tables6(**cfg)
        tup = synth.make_tuples6(T, n, gpu_id=rank)
        log(f"[rank {rank}] synthetic v6 tables ({len(T.ipc_keys)} ipcache, {len(T.pol_keys)} "
            f"policy) + {n} tuples in {time.time() - t0:.1f}s")
        e = Engine(device=local, **T.engine_config())
        synth.load_engine(e, T)
    else:
        T = synth.make_tables(**cfg)
        tup = synth.make_tuples(T, n, gpu_id=rank)
        if not cascade and not frames:
            # config 4: this rank's flowhash % world shard of the stream
            tup["sport"] = shard.assign_shard_sports(tup, world, rank, seed=synth.SEED + 0x5B0 + rank)
            assert (shard.shard_of(tup, world) == rank).all()
        if cascade:
            S = synth.make_services(T, cfg["n_services"])
            P4 = synth.make_prefilter4(T)
            tup = synth.add_prefilter_traffic(synth.add_service_traffic(tup, S, gpu_id=rank), P4,
                                              gpu_id=rank)
            del tup["hash"]  # skb->hash stand-in computed in the kernel from sport
        log(f"[rank {rank}] synthetic tables ({len(T.ipc_keys)} ipcache, {len(T.pol_keys)} policy"
            f"{', %d service-map entries' % len(S.keys) if S is not None else ''}) "
            f"+ {n} tuples in {time.time() - t0:.1f}s")
        ecfg = T.engine_config()
        if args.hot_slots:
            ecfg["hot_counter_slots"] = args.hot_slots
        if S is not None:
            ecfg["lb_max_entries"] = len(S.keys)
        e = Engine(device=local, **ecfg, schedule=args.schedule)
        synth.load_engine(e, T)
        if S is not None:
            synth.load_services(e, S)
        if cascade:
            synth.load_prefilter4(e, P4)
    t0 = time.time()
    e.commit()
    log(f"[rank {rank}] commit {time.time() - t0:.2f}s, checksum {e.checksum():#x}")
    if pf6 and args.host_tuples:
        d = {k: torch.from_numpy(np.ascontiguousarray(v, np.uint8)).pin_memory() for k, v in tup.items()}
        out = {"verdict": torch.empty(n, dtype=torch.uint8).pin_memory()}
    elif pf6:
        d = synth.packets6_to_device(tup, dev)
        out = {"verdict": torch.empty(n, dtype=torch.uint8, device=dev)}
    elif frames and args.host_tuples:
        # the frames in page-locked HOST memory (a receive ring), outputs
        # back into it: cgpu_classify_frames_host (PCIe-inclusive)
        fr = synth.frames_from_tuples(tup, stride=FRAME_STRIDE)
        d = {"data": torch.from_numpy(np.ascontiguousarray(fr["data"])).pin_memory(),
             "len": torch.from_numpy(np.ascontiguousarray(fr["len"], np.uint32).view(np.int32)).pin_memory(),
             "flags": torch.from_numpy(np.ascontiguousarray(fr["flags"], np.uint8)).pin_memory(),
             "ep": torch.from_numpy(np.ascontiguousarray(fr["ep"], np.uint16).view(np.int16)).pin_memory()}
        out = {"verdict": torch.empty(n, dtype=torch.int32).pin_memory(),
               "identity": torch.empty(n, dtype=torch.int32).pin_memory(), "stage": None}
    elif frames:
        fr = synth.frames_from_tuples(tup, stride=FRAME_STRIDE)
        d = synth.frames_to_device(fr, dev)
        out = {"verdict": torch.empty(n, dtype=torch.int32, device=dev),
               "identity": torch.empty(n, dtype=torch.int32, device=dev), "stage": None}
    elif args.host_tuples:
        # the batch in page-locked HOST memory, outputs back into it: every
        # step uploads the columns and downloads the verdicts through
        # cgpu_classify_v4_host / _v4_cascade_host / _v6_host (PCIe-inclusive;
        # DESIGN §6)
        view = {np.uint32: np.int32, np.uint16: np.int16, np.uint8: np.uint8, np.int32: np.int32}
        d = {k: torch.from_numpy(np.ascontiguousarray(v).view(view[v.dtype.type])).pin_memory()
             for k, v in tup.items()}
        out = {"verdict": torch.empty(n, dtype=torch.int32).pin_memory(),
               "identity": torch.empty(n, dtype=torch.int32).pin_memory(), "stage": None}
    else:
        d = synth.to_device(tup, dev)
        out = {"verdict": torch.empty(n, dtype=torch.int32, device=dev),
               "identity": torch.empty(n, dtype=torch.int32, device=dev), "stage": None}
        if ct:
            out["ct_ret"] = torch.empty(n, dtype=torch.uint8, device=dev)
        if ctlb:
            # the frame after the service step (lb4_xlate / lb6_xlate,
            # lb.h:700-775): part of the reference's result, written every step
            out["daddr"] = (torch.empty((n, 16), dtype=torch.uint8, device=dev) if ct6 else
                            torch.empty(n, dtype=torch.int32, device=dev))
            out["dport"] = torch.empty(n, dtype=torch.int16, device=dev)
    CT_NOW = 1000
    persist = args.ct_persist if (ct and not ctlb) else 0
    if args.ct_persist and not persist:
        raise SystemExit("--ct-persist applies to --config ct / ct6")
    CT_DT = 30  # seconds between steps in steady state (UDP / ICMP entries live 60 s)
    ct_k = [0]          # classify calls so far
    ct_ops = []         # ("cls", now) / ("gc", time), in order, for the restatement
    gc_log = []         # (entries deleted, host ms) per GC call
    delta = torch.zeros(e.counter_delta_bytes() // 8, dtype=torch.int64, device=dev)
    e.counter_bind(delta)
    stream = torch.cuda.current_stream()
    def check_layout(when):
        # replicas must map every policy key to the same counter slot before
        # their delta buffers are summed slot by slot
        lay = torch.tensor([e.counter_layout_checksum() & 0x7FFFFFFFFFFFFFFF], dtype=torch.int64,
                           device=dev)
        lo_, hi_ = lay.clone(), lay.clone()
        dist.all_reduce(lo_, op=dist.ReduceOp.MIN)
        dist.all_reduce(hi_, op=dist.ReduceOp.MAX)
        assert int(lo_) == int(hi_), f"counter slot layouts differ across ranks ({when})"

    if world > 1:
        check_layout("before warmup")
        shard.init_counter_comm(e, rank, world)

    def launch():
        now = CT_NOW + CT_DT * ct_k[0] if persist else CT_NOW
        if ct:
            ct_ops.append(("cls", now))
            ct_k[0] += 1
        if ctlb and ct6:
            e.classify_v6_ctlb(d, now, out=out, stream=stream)
        elif ct6:
            e.classify_v6_ct(d, now, out=out, stream=stream)
        elif ctlb:
            e.classify_v4_ctlb(d, now, out=out, stream=stream)
        elif ct:
            e.classify_v4_ct(d, now, out=out, stream=stream)
        elif pf6 and args.host_tuples:
            e.prefilter_host(d["saddr"], d["daddr"], d["flags"], v6=True, out=out["verdict"], stream=stream)
        elif pf6:
            e.prefilter_v6(d["saddr"], d["daddr"], d["flags"], out=out["verdict"], stream=stream)
        elif cascade and args.host_tuples:
            e.classify_v4_lb_host(d, out=out, stream=stream, xdp=True)
        elif cascade:
            e.classify_v4_cascade(d, out=out, stream=stream)
        elif v6 and args.host_tuples:
            e.classify_v6_host(d, out=out, stream=stream)
        elif v6:
            e.classify_v6(d, out=out, stream=stream)
        elif frames and args.host_tuples:
            e.classify_frames_host(d, out=out, stream=stream)
        elif frames:
            e.classify_frames(d, out=out, stream=stream)
        elif args.host_tuples:
            e.classify_v4_host(d, out=out, stream=stream)
        else:
            e.classify_v4(d, out=out, stream=stream)

    def flush_ct():
        if ct6:
            e.ct6_flush()
        elif ct:
            e.ct4_flush()

    def gc_ct():
        # ctmap.GC RemoveExpired at the coming step's time, on the device map
        tm = CT_NOW + CT_DT * ct_k[0]
        g0 = time.perf_counter()
        dl = e.ct6_gc(tm) if ct6 else e.ct4_gc(tm)
        gc_log.append((dl, 1e3 * (time.perf_counter() - g0)))
        ct_ops.append(("gc", tm))

    def step(ev=None):
        if persist:
            if ct_k[0] and ct_k[0] % persist == 0:
                gc_ct()
        elif ct:
            flush_ct()  # every step starts from an empty conntrack map
        if ev is not None:
            ev[0].record(stream)
        launch()
        if ev is not None:
            ev[1].record(stream)
        shard.reduce_counters(e, world, stream)  # RCCL over xGMI: u64 SUM, order-independent
        e.counter_fold(stream)

    for _ in range(args.warmup):
        step()
    # the control plane's periodic slot rebalance (cgpu_counters_rebalance):
    # after warmup traffic the most-hit keys own the LDS counter slots; every
    # rank holds the same folded totals, so every rank picks the same layout
    moved = None
    if not args.no_rebalance and not pf6 and args.warmup:
        torch.cuda.synchronize()
        moved = e.counters_rebalance()
        if world > 1:
            # the rebalance moved slots again: every rank must have moved them
            # the same way before the timed steps' slot-wise sums
            check_layout("after counters_rebalance")
        step()
    evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
           for _ in range(args.steps)]
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t_start = time.perf_counter()
    for k in range(args.steps):
        step(evs[k])
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t_start
    kern_ms = sum(a.elapsed_time(b) for a, b in evs) / args.steps
    if world > 1:
        tt = torch.tensor([elapsed, kern_ms], dtype=torch.float64, device=dev)
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        elapsed, kern_ms = float(tt[0]), float(tt[1])
    ms_per_step = 1e3 * elapsed / args.steps
    value = world * n * args.steps / elapsed / 1e6

    allreduce_ok = None
    if world > 1:
        # the shipped collective against torch's SUM of the same local deltas
        # (one untimed step): every rank must hold the sum of all ranks
        if ct and not persist:
            flush_ct()
        torch.cuda.synchronize()
        delta.zero_()
        launch()
        torch.cuda.synchronize()
        local = delta.clone()
        shard.reduce_counters(e, world, stream)
        dist.all_reduce(local, op=dist.ReduceOp.SUM)
        torch.cuda.synchronize()
        ok = torch.tensor([int(torch.equal(local, delta))], dtype=torch.int64, device=dev)
        dist.all_reduce(ok, op=dist.ReduceOp.MIN)
        allreduce_ok = bool(int(ok))
        e.counter_fold(stream)

    # the replicated map contents (cgpu_table_checksum) must agree across
    # ranks, and so must the counter slot layout the timed sums relied on
    if world > 1:
        check_layout("after the timed steps")
        cs = torch.tensor([e.checksum() & 0x7FFFFFFFFFFFFFFF], dtype=torch.int64, device=dev)
        lo, hi = cs.clone(), cs.clone()
        dist.all_reduce(lo, op=dist.ReduceOp.MIN)
        dist.all_reduce(hi, op=dist.ReduceOp.MAX)
        assert int(lo) == int(hi), "replicated tables differ across ranks"

    result = None
    # the CPU baseline is an N=1 figure (rank 0 alone); at N > 1 the
    # restatement runs once, for the parity check of rank 0's batch only
    skip_cpu = args.no_cpu_baseline or world > 1
    if rank == 0 and args.no_parity:
        result = {"metric": METRIC, "value": round(value, 2), "unit": "Mpps", "n_gpus": world,
                  "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(ms_per_step, 4),
                  "config": {"workload": WORKLOADS[args.config], "kernel_ms": round(kern_ms, 4),
                             "parity_vs_oracle": None, "note": "--no-parity profiling pass"}}
    elif rank == 0:
        sys.path.insert(0, os.path.join(ROOT, "oracle"))
        from oracle import Oracle  # CPU restatement: checker + CPU baseline only

        threads = args.cpu_threads or min(int(os.environ.get("OMP_NUM_THREADS", "0")) or
                                          os.cpu_count(), os.cpu_count())
        if pf6:
            o = Oracle(**P.oracle_config())
            synth.load_prefilter6(o, P)
        elif ct:
            o = Oracle(**T.oracle_config())
            synth.load_oracle(o, T)
            synth.load_lxc(o, seclabels)
            o.ct_set_max(ct_max)
            o.ct6_set_max(ct_max)
            if S is not None:
                (synth.load_services6 if ct6 else synth.load_services)(o, S)
        else:
            o = Oracle(**T.oracle_config())
            synth.load_oracle(o, T)
            if S is not None:
                synth.load_services(o, S)
            if cascade:
                synth.load_prefilter4(o, P4)
        def cpu_run(sl):
            if pf6:
                return o.prefilter_v6(tup["saddr"][sl], tup["daddr"][sl], tup["flags"][sl],
                                      nthreads=threads)
            if cascade:
                return o.classify_v4_cascade({k: v[sl] for k, v in tup.items()}, nthreads=threads)
            if v6:
                return o.classify_v6({k: v[sl] for k, v in tup.items()}, nthreads=threads)
            if frames:
                return o.classify_frames({k: v[sl] for k, v in fr.items()}, nthreads=threads)
            return o.classify_v4({k: v[sl] for k, v in tup.items()}, nthreads=threads)

        cpu = None
        cpu_thr = None
        if ct:
            # the stateful restatement (oracle/cgpu_oracle.c or_classify_v{4,6}_ct{,lb}),
            # threaded over shards with a conntrack map per shard (Oracle.sharded)
            meth = f"classify_v{6 if ct6 else 4}_ct{'lb' if ctlb else ''}"
            sub = np.arange(n)
            if ctlb:
                # parity: the sequential restatement over the whole batch (a
                # service's connections are tied to its backends' pairs, so no
                # pair partition is exact); the CPU baseline: the same code
                # threaded RSS-style by connection (shard.conn_shard_of),
                # checked against the sequential result
                o.probe_split()
                c0 = time.perf_counter()
                r_ = getattr(o, meth)(tup, CT_NOW)
                seq_s = time.perf_counter() - c0
                split = o.probe_split()
                first = (r_["verdict"], r_["ct_ret"], r_["identity"], r_["stage"], r_["probes"])
                x0 = (r_["xdaddr"], r_["xdport"])
                if not skip_cpu:
                    o2 = Oracle(**T.oracle_config())
                    synth.load_oracle(o2, T)
                    synth.load_lxc(o2, seclabels)
                    o2.ct_set_max(ct_max)
                    o2.ct6_set_max(ct_max)
                    (synth.load_services6 if ct6 else synth.load_services)(o2, S)
                    # threaded over an EXACT partition: the connected components
                    # of the address pairs a packet can touch through any
                    # backend of its service (shard.svc_component_shard_of)
                    p0 = time.perf_counter()
                    comp = shard.svc_component_shard_of(tup, S.keys, S.vals, 4 * threads,
                                                        0 if ct6 else L.IPV4_LOOPBACK)
                    part_s = time.perf_counter() - p0
                    rs, c_el = o2.sharded(meth, tup, CT_NOW, comp, threads)
                    same = all(np.array_equal(rs[k], r_[k]) for k in
                               ("verdict", "ct_ret", "identity", "stage", "xdaddr", "xdport"))
                    cpu = {"value": round(n / c_el / 1e6, 3), "unit": "Mpps", "cores": threads,
                           "kind": "port",
                           "sample": (f"rank-0 batch, all {n} packets from an empty map; "
                                      f"oracle/cgpu_oracle.c or_{meth} threaded over {4 * threads} "
                                      f"shards of an exact partition (shard.svc_component_shard_of: "
                                      f"connected components of the address pairs reachable through "
                                      f"any backend, {part_s:.1f}s to compute, untimed), a conntrack "
                                      f"map per shard, on {threads} threads, {c_el:.2f}s wall of the "
                                      f"parallel section; results equal to the sequential run's: "
                                      f"{same}; host: {host_cpu()}")}
                    cpu_thr = {"value": round(n / seq_s / 1e6, 3), "unit": "Mpps", "cores": 1,
                               "kind": "port, sequential",
                               "sample": (f"the same code on 1 thread over the whole batch in order "
                                          f"(the parity reference), {seq_s:.1f}s")}
            elif persist:
                # steady state: the same batch replayed in the same order of
                # steps and GCs (ct_ops) over pair-shard views whose maps
                # persist; the last step's results are the parity reference
                o.probe_split()
                first, walls, odels = o.sharded_steps(meth, tup, shard.ct_shard_of(tup, 4 * threads),
                                                      threads, ct_ops)
                split = o.probe_split()
                cls_w = [w for (op_, _), w in zip(ct_ops, walls) if op_ == "cls"]
                c_el = float(np.median(cls_w))
                gc_same = odels == [dl for dl, _ in gc_log]
                # probes of the last batch only (probe_split counted all of them)
                n_cls = len(cls_w)
                split = {k_: v_ // n_cls for k_, v_ in split.items()}
                if not skip_cpu:
                    cpu = {"value": round(n / c_el / 1e6, 3), "unit": "Mpps", "cores": threads,
                           "kind": "port",
                           "sample": (f"rank-0 batch, all {n} packets per step, {n_cls} steps replayed "
                                      f"with the same times and {len(odels)} GCs over persistent "
                                      f"conntrack maps per address-pair shard (Oracle.sharded_steps, "
                                      f"{4 * threads} shards) on {threads} threads; median "
                                      f"{c_el:.2f}s wall per batch; host: {host_cpu()}")}
            else:
                # address pairs are independent conntrack groups (every key a
                # packet touches carries its pair): the pair-sharded run is
                # exactly the sequential result for the whole batch
                o.probe_split()
                first, c_el = o.sharded(meth, tup, CT_NOW, shard.ct_shard_of(tup, 4 * threads),
                                        threads)
                split = o.probe_split()
                if not skip_cpu:
                    cpu = {"value": round(n / c_el / 1e6, 3), "unit": "Mpps", "cores": threads,
                           "kind": "port",
                           "sample": (f"rank-0 batch, all {n} packets from an empty map; "
                                      f"oracle/cgpu_oracle.c or_{meth} (sequential conntrack + LPM "
                                      f"trie + open hash per address-pair shard: "
                                      f"shard.ct_shard_of, {4 * threads} shards, a conntrack map per "
                                      f"shard) on {threads} threads, {c_el:.2f}s wall of the parallel "
                                      f"section; host: {host_cpu()}")}
        elif not skip_cpu:
            cpu_run(slice(0, min(n, 1 << 20)))  # warm the tables' pages before timing
        # the median of 3 timed runs (the first also yields the reference result)
        runs = []
        if not ct:
            o.probe_split()
        def run_full():
            if pf6:
                return o.prefilter_v6(tup["saddr"], tup["daddr"], tup["flags"], nthreads=threads)
            if cascade:
                return o.classify_v4_cascade(tup, nthreads=threads)
            if v6:
                return o.classify_v6(tup, nthreads=threads)
            if frames:
                return o.classify_frames(fr, nthreads=threads)
            return o.classify_v4(tup, nthreads=threads)

        for rep in range(0 if ct else 3):
            c0 = time.perf_counter()
            res = run_full()
            runs.append(time.perf_counter() - c0)
            if rep == 0:
                first = res
                split = o.probe_split()
            if skip_cpu:
                break
        if ct:
            v0, cr0, i0, _, probes = first
            if persist:
                probes = sum(split.values())
        elif pf6:
            c_el = float(np.median(runs))
            v0, probes = first
        else:
            c_el = float(np.median(runs))
            v0, i0, _, probes = first
        n_cpu = n
        if not skip_cpu and not ct:
            what = {"pf6": "oracle/cgpu_oracle.c prefilter (kernel-like LPM trie + hash)",
                    "cascade": ("oracle/cgpu_oracle.c or_classify_v4_cascade: XDP check_v4 (LPM trie + "
                                "hash + endpoint hash) | lb4_local, then LPM trie + open hash"),
                    "v6": "oracle/cgpu_oracle.c IPv6 LPM trie + open hash",
                    "frames": "oracle/cgpu_oracle.c frame parse + LPM trie + open hash"}.get(
                args.config, "oracle/cgpu_oracle.c (kernel-like LPM trie + open hash)")
            cpu = {"value": round(n / c_el / 1e6, 3), "unit": "Mpps", "cores": threads,
                   "kind": "port",
                   "sample": f"rank-0 batch, all {n} tuples, {args.config} tables; {what}, "
                             f"{threads} threads, median of {len(runs)} runs "
                             f"{'/'.join(f'{x:.2f}' for x in runs)} s; host: {host_cpu()}"}
        cpu_opt = None
        if not skip_cpu and not ct:
            # BASELINE.md §2's optimized CPU path: the same restatement with
            # the ipcache (and the prefilter's deny LPMs) as a DIR-24-8 /
            # multibit trie (oracle/fast_lpm.h), checked equal to the port
            o.set_fast(True)
            runs_o = []
            for rep in range(3):
                c0 = time.perf_counter()
                r_o = run_full()
                runs_o.append(time.perf_counter() - c0)
                if rep == 0:
                    same_o = bool(np.array_equal(r_o[0], v0 if pf6 else first[0]) and
                                  (pf6 or np.array_equal(r_o[1], first[1])))
            o.set_fast(False)
            el_o = float(np.median(runs_o))
            cpu_opt = {"value": round(n / el_o / 1e6, 3), "unit": "Mpps", "cores": threads,
                       "kind": "optimized",
                       "sample": (f"rank-0 batch, all {n} tuples; the restatement with the "
                                  f"{'prefilter deny LPM' if pf6 else 'ipcache'} as a DIR-24-8 (IPv4) / "
                                  f"multibit trie with per-/64 lists (IPv6) (oracle/fast_lpm.h, "
                                  f"BASELINE.md §2), {threads} threads, median of 3 runs "
                                  f"{'/'.join(f'{x:.2f}' for x in runs_o)} s; results equal to the "
                                  f"port's: {same_o}; host: {host_cpu()}")}
        if ct:
            parity = bool(np.array_equal(out["verdict"].cpu().numpy(), v0) and
                          np.array_equal(out["ct_ret"].cpu().numpy(), cr0) and
                          np.array_equal(out["identity"].cpu().numpy().view(np.uint32), i0))
            if ctlb:
                xd = out["daddr"].cpu().numpy()
                parity = parity and np.array_equal(xd if ct6 else xd.view(np.uint32), x0[0]) and \
                    np.array_equal(out["dport"].cpu().numpy().view(np.uint16), x0[1])
        else:
            parity = bool(np.array_equal(out["verdict"].cpu().numpy(), v0))
            if not pf6:
                parity = parity and np.array_equal(out["identity"].cpu().numpy().view(np.uint32), i0)
        probes_per = probes / n_cpu
        b_in, b_out = ((B_IN_PF6, B_OUT_PF6) if pf6 else (B_IN_FRAMES, B_OUT) if frames
                       else (B_IN_CT6 + (4 if ctlb else 0), B_OUT_CT) if ct6 else (B_IN_CT + (4 if ctlb else 0), B_OUT_CT) if ct
                       else (B_IN_V6, B_OUT) if v6
                       else (B_IN + (2 if cascade else 0), B_OUT))
        b_alg = b_in + b_out + 64.0 * probes_per
        achieved = b_alg * n / (kern_ms * 1e-3) / 1e9
        traffic, traffic_note, traffic_dom = pmc_traffic(args)
        tb = e.table_bytes()
        roof = roofline(n_cpu, kern_ms, b_in, b_out, probes, split, tb, ct6 or v6 or pf6, traffic_dom)
        # the same floor with every table at the REFERENCE's own map footprint
        # (entries x (key + value) bytes of the BPF map): a larger engine
        # layout moves its lookups to a slower tier and so raises the floor;
        # priced at the reference's bytes the floor is the lower of the two
        ref_tb = dict(tb)
        if not pf6:
            ref_tb.update(ipcache=len(T.ipc_keys) * (24 + 8), policy=len(T.pol_keys) * (8 + 24))
            if S is not None:
                ref_tb.update(lb4=len(S.keys) * (8 + 12), lb6=len(S.keys) * (20 + 24))
            if cascade:
                ref_tb.update(prefilter=(len(P4.dyn4) + len(P4.fix4)) * (8 + 4),
                              endpoint=len(P4.ep_keys) * (20 + 24))
            if ct:
                ce = int(e.ct6_count() if ct6 else e.ct4_count())
                ref_tb.update(ct4=ce * (14 + 56), ct6=ce * (38 + 56))
        roof_ref = roofline(n_cpu, kern_ms, b_in, b_out, probes, split, ref_tb, ct6 or v6 or pf6, traffic_dom)
        if roof is not None and roof_ref is not None:
            roof["frac_at_reference_footprint"] = roof_ref["frac"]
            roof["bound_at_reference_footprint"] = roof_ref["bound"]
            roof["reference_footprint_bytes"] = {k: ref_tb[k] for k in ("ipcache", "policy", "lb4", "lb6",
                                                                       "prefilter", "endpoint", "ct4", "ct6")
                                                 if k in ref_tb and ref_tb[k] != tb.get(k)}
        conf = {"workload": WORKLOADS[args.config], "tuples_per_gpu": n,
                "parallelism": f"shard{world}", "kernel_ms": round(kern_ms, 4),
                "stream_tuples_per_step": world * n, "stream_tuples_timed": world * n * args.steps,
                "counter_reduce": ("cgpu_counters_allreduce (RCCL u64 SUM)" if world > 1 else "none (1 rank)"),
                "allreduce_check_vs_torch_sum": allreduce_ok,
                "counter_slots": ("class-based" if moved is None else
                                  f"popularity-rebalanced after warmup ({moved} keys moved)"),
                "probes_per_tuple": round(probes_per, 4), "b_alg_per_tuple": round(b_alg, 2),
                "parity_vs_oracle": parity}
        if args.schedule:
            conf["schedule"] = args.schedule
        if args.host_tuples:
            bw = link_rates(torch, dev)
            # bytes up / down per tuple (frames: the 64-byte slot + len, flags, ep)
            per_in, per_out = b_in, b_out
            conf.update(host_tuples=True,
                        pcie_measured_gbs=bw,
                        numa={"gpu": gpu_numa_node(torch, dev),
                              "inputs": numa_nodes(d["data" if frames else "saddr"]),
                              "verdict": numa_nodes(out["verdict"]),
                              "identity": numa_nodes(out["identity"]) if "identity" in out else None},
                        ingest_bound_mpps=round(min(bw["h2d"] * 1e3 / per_in, bw["d2h"] * 1e3 / per_out,
                                                    bw["both"] * 1e3 / (per_in + per_out)), 1),
                        hbm_resident_roofline=roof,
                        note=(f"PCIe-inclusive: the {'frames (64-B slots + len, flags, ep' if frames else 'columns ('}"
                              f"{per_in} B/tuple) go up and the outputs ({per_out} B/tuple) come down every "
                              "step through the device staging chunks; ingest_bound_mpps = the measured link "
                              "rates over those bytes (each direction alone, and both directions at once "
                              "over their sum). The HBM-resident rate is the default line (no --host-tuples)"))
            # the host line is bound by the link: each direction's bytes at
            # its rate alone, and the bytes of both at the measured rate of
            # the two directions at once; the largest floor binds
            t_s = ms_per_step * 1e-3
            t_up, t_down = n * per_in / (bw["h2d"] * 1e9), n * per_out / (bw["d2h"] * 1e9)
            t_both = n * (per_in + per_out) / (bw["both"] * 1e9)
            t_floor = max(t_up, t_down, t_both)
            roof = {"bound": "link", "achieved": round(n * (per_in + per_out) / t_s / 1e9, 2),
                    "peak": round(n * (per_in + per_out) / t_floor / 1e9, 2), "unit": "GB/s",
                    "frac": round(t_floor / t_s, 4),
                    "frac_one_direction": round(max(t_up, t_down) / t_s, 4),
                    "components": {"h2d": {"gbs": bw["h2d"], "frac": round(t_up / t_s, 4)},
                                   "d2h": {"gbs": bw["d2h"], "frac": round(t_down / t_s, 4)},
                                   "both": {"gbs": bw["both"], "frac": round(t_both / t_s, 4)}}}
        if pf6:
            conf.update(dyn6_prefixes=len(P.dyn6), fix6_prefixes=len(P.fix6),
                        endpoints=len(P.ep6))
        else:
            conf.update(ipcache_prefixes=int(len(T.ipc_keys)), policy_entries=int(len(T.pol_keys)))
            if S is not None:
                conf.update(services=int(len(S.vip)), lb_map_entries=int(len(S.keys)))
            if cascade:
                conf.update(prefilter_dyn4=int(len(P4.dyn4)), prefilter_fix4=int(len(P4.fix4)),
                            local_endpoints=int(len(P4.ep_keys)),
                            xdp_drop_frac_of_ingress=round(float(
                                (v0 == -4097).sum() / max(1, int(((tup["flags"] & 1) == 0).sum()))), 4))
            if ct:
                ctr = out["ct_ret"].cpu().numpy()
                conf.update(ct_max=ct_max,
                            ct_entries_after_step=int(e.ct6_count() if ct6 else e.ct4_count()),
                            parity_packets=int(len(sub)),
                            ct_state_frac={s_: round(float((ctr == c_).mean()), 4) for s_, c_ in
                                           (("new", 0), ("established", 1), ("reply", 2),
                                            ("related", 3), ("none", 255))},
                            ops_per_packet_note="probes = ipcache + policy probes + CT map "
                                                "lookups/updates/deletes of the reference "
                                                "(+ service lookups), counted by the restatement "
                                                "over the whole batch")
                if persist:
                    timed_gc = gc_log[-(args.steps // persist + 1):]
                    conf.update(ct_persist={
                        "gc_every_steps": persist, "seconds_per_step": CT_DT,
                        "steps_total": ct_k[0], "gc_calls": len(gc_log),
                        "gc_deleted": [dl for dl, _ in gc_log],
                        "gc_deleted_equal_restatement": gc_same,
                        "gc_ms_per_call": round(float(np.median([ms for _, ms in gc_log])), 3) if gc_log else None,
                        "gc_ms_in_timed_steps": round(sum(ms for _, ms in timed_gc), 3),
                        "ct_stats_after": e.ct_stats(ct6),
                        "note": ("the same 64M-packet batch every step, 30 s apart, so UDP / ICMP / "
                                 "SYN-only entries (60 s) expire and are re-created while TCP "
                                 "connections stay established; kernel_ms is the classify alone, "
                                 "ms_per_step includes the GC calls (device GC, one host read)")})
        result = {
            "metric": (f"Mpps classified from host-resident {'raw frames' if frames else 'batches'} (PCIe-inclusive)"
                       if args.host_tuples
                       else METRIC if not pf6 else "Mpps XDP IPv6 prefilter verdicts; % HBM roofline"),
            "value": round(value, 2), "unit": "Mpps", "n_gpus": world,
            "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(ms_per_step, 4),
            "higher_is_better": True, "scaling": "weak", "vs_baseline": None,
            "dtype": "u8" if pf6 else "u32",
            "data": "synthetic (seeded PCG64 tables + tuples, SURVEY §8d)",
            "config": conf,
            "roofline": dict(roof or {"bound": None, "note": "profiles/ceilings.json absent"},
                             traffic=traffic, traffic_source=traffic_note,
                             traffic_dominant_kernel=traffic_dom,
                             hbm_side_frac=(round(traffic / (kern_ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 4)
                                            if traffic else None),
                             # the round-1..4 model, kept for comparison: 64 B per
                             # reference lookup against the 8 TB/s HBM peak; it is
                             # not a bound (the tables are L2 / MALL hits), so
                             # it can exceed 1
                             b_alg={"achieved": round(achieved, 1), "peak": HBM_PEAK_GBS,
                                    "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBS, 4),
                                    "basis": "B_alg (columns + 64 B per reference map lookup)"}),
            "cpu_baseline": cpu,
            "cpu_baseline_optimized": cpu_opt,
        }
        if cpu_thr is not None:
            result["cpu_baseline_sequential"] = cpu_thr
        if not parity:
            log("WARNING: GPU verdicts differ from the restatement")
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()
    e.close()
    if rank == 0:
        print(json.dumps(result), flush=True)


def bench_mapstate(args, rank, world, local):
    """one step = cgpu_l3_compile of every (endpoint,
    identity) pair (upload of the interned tables, the device walk, the
    allow matrix back).  Ranks take disjoint endpoint slices (weak: each
    rank compiles its own 100 endpoints against all identities)."""
    import numpy as np
    import torch

    from cilium_amd import synth
    from cilium_amd.engine import Engine

    torch.cuda.set_device(local)
    t0 = time.time()
    repo, eps, ids = synth.make_l3_workload(seed=synth.SEED + rank)
    prog = repo.compile()
    log(f"[rank {rank}] {len(repo.rules)} rules ({len(prog.clauses)} clauses, {len(prog.selectors)} "
        f"selectors), {len(eps)} endpoints x {len(ids)} identities in {time.time() - t0:.1f}s")
    e = Engine(device=local)
    # the label arrays are interned once, as the agent's identity cache
    # holds them; a step is the compile of every pair
    eps_i, ids_i = prog.label_sets(eps), prog.label_sets(ids)
    for _ in range(args.warmup):
        allow = e.l3_compile(prog, eps_i, ids_i)
    t_start = time.perf_counter()
    for _ in range(args.steps):
        allow = e.l3_compile(prog, eps_i, ids_i)
    elapsed = time.perf_counter() - t_start
    pairs = len(eps) * len(ids)
    result = None
    if rank == 0:
        sys.path.insert(0, os.path.join(ROOT, "oracle"))
        from oracle import Oracle
        c0 = time.perf_counter()
        ref = Oracle.l3_compile(prog, eps[:2], ids)
        c_el = time.perf_counter() - c0
        parity = bool(np.array_equal(allow[:2], ref))
        value = world * pairs * args.steps / elapsed / 1e6
        # bytes the walk must read per pair: the identity's labels (12 B
        # each) and the allow byte; the program and endpoint labels stay
        # in cache across pairs
        nlab = sum(len(x) for x in ids) / len(ids)
        b_pair = 12.0 * nlab + 1.0
        achieved = b_pair * pairs / (elapsed / args.steps) / 1e9
        result = {
            "metric": "M (endpoint, identity) L3 policy decisions/s (computeDesiredL3PolicyMapEntries)",
            "value": round(value, 2), "unit": "M decisions/s", "n_gpus": world, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": round(1e3 * elapsed / args.steps, 3),
            "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "u32",
            "data": "synthetic (seeded repository + label sets)",
            "config": {"workload": WORKLOADS["mapstate"], "rules": len(repo.rules),
                       "clauses": int(len(prog.clauses)), "selectors": int(len(prog.selectors)),
                       "endpoints": len(eps), "identities": len(ids), "parity_vs_oracle": parity,
                       "allowed_frac": {"ingress": round(float((allow & 1).mean()), 4),
                                        "egress": round(float((allow & 2).astype(bool).mean()), 4)},
                       "note": "host-pointer control-plane call: the step includes the table "
                               "upload and the allow-matrix download"},
            "roofline": {"bound": "hbm", "achieved": round(achieved, 2), "peak": HBM_PEAK_GBS,
                         "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBS, 5), "traffic": None},
            "cpu_baseline": {"value": round(2 * len(ids) / c_el / 1e6, 4), "unit": "M decisions/s",
                             "cores": 1, "kind": "port",
                             "sample": f"2 endpoints x {len(ids)} identities; oracle/cgpu_oracle.c "
                                       f"or_l3_compile, 1 thread, {c_el:.2f}s wall"},
        }
    e.close()
    if rank == 0:
        print(json.dumps(result), flush=True)


if __name__ == "__main__":
    main()
