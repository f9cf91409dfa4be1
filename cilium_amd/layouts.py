"""Reference byte layouts of the map keys/values on the classification path.

These are the exact layouts the reference datapath and its Go map wrappers
exchange through bpf(2); the C ABI (include/cgpu.h) takes the same bytes so a
cgo caller can pass ``unsafe.Pointer`` straight through.

* ``policy_key`` 8 B / ``policy_entry`` 24 B — bpf/lib/common.h:180-193,
  Go mirror pkg/maps/policymap/policymap.go:63-80.  ``egress`` is the byte
  holding the ``egress:1, pad:7`` bitfield (bit 0 = egress on little endian).
* ``ipcache_key`` 24 B / ``remote_endpoint_info`` 8 B — bpf/lib/maps.h:135-148,
  bpf/lib/common.h:175-178, Go pkg/maps/ipcache/ipcache.go:54-61,132-135.
  ``prefixlen`` counts the 32 static bits (pad[3] + family) plus the IP bits
  (bpf/lib/eps.h:48-52, ipcache.go:72-98).
* ``lpm_v4_key`` 8 B / ``lpm_v6_key`` 20 B — bpf/lib/xdp.h:23-31, Go
  pkg/maps/cidrmap/cidrmap.go:49-52 (``cidrKey`` truncated to 4 + AddrSize).
* ``endpoint_key`` 20 B — bpf/lib/common.h:147-160.
* ``metrics`` {reason, dir} -> {count, bytes} — bpf/lib/common.h:195-206.
* ``lb4_key`` 8 B / ``lb4_service`` 12 B — bpf/lib/common.h:427-439, Go
  pkg/maps/lbmap/ipv4.go:78-190 (key port, value port / rev_nat / weight in
  network order after ToNetwork; slave and count stay host order).
"""
from __future__ import annotations

import ipaddress
import socket
import struct

import numpy as np

POLICY_KEY = np.dtype([("sec_label", "<u4"), ("dport", "<u2"), ("protocol", "u1"),
                       ("egress", "u1")])
POLICY_ENTRY = np.dtype([("proxy_port", "<u2"), ("pad", "<u2", (3,)), ("packets", "<u8"),
                         ("bytes", "<u8")])
IPCACHE_KEY = np.dtype([("prefixlen", "<u4"), ("pad", "u1", (3,)), ("family", "u1"),
                        ("ip", "u1", (16,))])
REMOTE_ENDPOINT_INFO = np.dtype([("sec_label", "<u4"), ("tunnel_endpoint", "<u4")])
LPM_V4_KEY = np.dtype([("prefixlen", "<u4"), ("addr", "u1", (4,))])
LPM_V6_KEY = np.dtype([("prefixlen", "<u4"), ("addr", "u1", (16,))])
ENDPOINT_KEY = np.dtype([("ip", "u1", (16,)), ("family", "u1"), ("pad4", "u1"),
                         ("pad5", "<u2")])

assert POLICY_KEY.itemsize == 8 and POLICY_ENTRY.itemsize == 24
assert IPCACHE_KEY.itemsize == 24 and REMOTE_ENDPOINT_INFO.itemsize == 8
LB4_KEY = np.dtype([("address", "<u4"), ("dport", "<u2"), ("slave", "<u2")])
LB4_SERVICE = np.dtype([("target", "<u4"), ("port", "<u2"), ("count", "<u2"),
                        ("rev_nat_index", "<u2"), ("weight", "<u2")])
assert LB4_KEY.itemsize == 8 and LB4_SERVICE.itemsize == 12
# struct lb6_key / lb6_service, bpf/lib/common.h:408-420 (packed)
LB6_KEY = np.dtype([("address", "u1", 16), ("dport", "<u2"), ("slave", "<u2")])
LB6_SERVICE = np.dtype([("target", "u1", 16), ("port", "<u2"), ("count", "<u2"),
                        ("rev_nat_index", "<u2"), ("weight", "<u2")])
assert LB6_KEY.itemsize == 20 and LB6_SERVICE.itemsize == 24
assert LPM_V4_KEY.itemsize == 8 and LPM_V6_KEY.itemsize == 20
assert ENDPOINT_KEY.itemsize == 20

# bpf/lib/common.h:139-140
ENDPOINT_KEY_IPV4 = 1
ENDPOINT_KEY_IPV6 = 2
# bpf/lib/eps.h:48-52: 8 * (sizeof(ipcache_key) - sizeof(bpf_lpm_trie_key) - 16)
IPCACHE_STATIC_PREFIX = 32

# reserved identities, bpf/node_config.h:34-38 / pkg/identity
HOST_ID, WORLD_ID, CLUSTER_ID, HEALTH_ID, INIT_ID = 1, 2, 3, 4, 5
# drop reasons, bpf/lib/common.h:237-269
DROP_POLICY = -133
DROP_CT_UNKNOWN_PROTO = -137
DROP_FRAG_NOSUPPORT = -157
XDP_DROP, XDP_PASS = 1, 2
# cgpu_classify_v4_cascade (config 5 whole): an ingress tuple the netdev's XDP
# prefilter dropped (bpf_xdp.c:97-121) -- the engine's own code, like
# DROP_SNAPLEN: the XDP program returns XDP_DROP and records no drop reason
VERDICT_XDP_DROP = -4097
STAGE_XDP_DROP = 8
METRIC_INGRESS, METRIC_EGRESS = 1, 2
# CT direction (bpf/lib/common.h:327-328); policy_key.egress = !dir
CT_EGRESS, CT_INGRESS = 0, 1

PROTO_ICMP, PROTO_TCP, PROTO_UDP = 1, 6, 17

DROP_NO_SERVICE = -158
TC_ACT_OK, TC_ACT_REDIRECT = 0, 7
# IPV4_LOOPBACK (bpf/node_config.h:45), network-order u32 as written
IPV4_LOOPBACK = 0x1ffff50a
# cgpu_lb4_select modes and LXC result codes (include/cgpu.h)
LB_NETDEV, LB_LXC = 0, 1
LB_NONE, LB_XLATED, LB_XLATED_LOOPBACK = 0, 1, 2
LB_L3, LB_L4 = 1, 2

# tuple flag bits of the classify SoA
F_EGRESS = 1
F_FRAGMENT = 2
# prefilter packet flags
PKT_OK, PKT_TRUNCATED, PKT_NOT_IP = 0, 1, 2

# conntrack: struct ipv4_ct_tuple (packed, 14 B) and struct
# ct_entry (56 B), bpf/lib/common.h:359-408; the map cilium_ct4_global
CT4_TUPLE = np.dtype([("daddr", "<u4"), ("saddr", "<u4"), ("dport", "<u2"), ("sport", "<u2"),
                      ("nexthdr", "u1"), ("flags", "u1")])
assert CT4_TUPLE.itemsize == 14
# struct ipv6_ct_tuple (common.h:338-346), packed, 38 B
CT6_TUPLE = np.dtype([("daddr", "u1", 16), ("saddr", "u1", 16), ("dport", "<u2"), ("sport", "<u2"),
                      ("nexthdr", "u1"), ("flags", "u1")])
assert CT6_TUPLE.itemsize == 38
CT_ENTRY = np.dtype([("rx_packets", "<u8"), ("rx_bytes", "<u8"), ("tx_packets", "<u8"),
                     ("tx_bytes", "<u8"), ("lifetime", "<u4"), ("bits", "<u2"),
                     ("rev_nat_index", "<u2"), ("slave", "<u2"), ("tx_flags_seen", "u1"),
                     ("rx_flags_seen", "u1"), ("src_sec_id", "<u4"), ("last_tx_report", "<u4"),
                     ("last_rx_report", "<u4")])
assert CT_ENTRY.itemsize == 56
# ct_entry bit field (common.h:385-390)
CTB_RX_CLOSING, CTB_TX_CLOSING, CTB_NAT46, CTB_LB_LOOPBACK, CTB_SEEN_NON_SYN = 1, 2, 4, 8, 16
# ct_lookup4 results (common.h:331-336); 255 = ct_lookup4 failed (DROP_CT_UNKNOWN_PROTO)
CT_NEW, CT_ESTABLISHED, CT_REPLY, CT_RELATED, CT_NONE = 0, 1, 2, 3, 255
TUPLE_F_OUT, TUPLE_F_IN, TUPLE_F_RELATED = 0, 1, 2
DROP_CT_CREATE_FAILED = -155
TCP_FIN, TCP_SYN, TCP_RST, TCP_PSH, TCP_ACK = 0x01, 0x02, 0x04, 0x08, 0x10
CT_MAX_GLOBAL = 1000000  # pkg/maps/ctmap/ctmap.go:101 MapNumEntriesGlobal


def ct_sorted(keys: np.ndarray, vals: np.ndarray):
    """Dump of a CT map in a canonical order (key bytes) for comparisons."""
    kb = np.ascontiguousarray(keys).view(np.uint8).reshape(len(keys), keys.dtype.itemsize)
    order = np.lexsort(kb.T[::-1])
    return keys[order], vals[order]


# per-endpoint identity of the endpoint program (cgpu_lxc_info, include/cgpu.h;
# lxc_config.h LXC_MAC / LXC_IPV4 / LXC_IP, bpf/lib/lxc.h:31-89)
LXC_INFO = np.dtype([("mac", "u1", (6,)), ("verify", "u1"), ("pad", "u1"), ("ipv4", "<u4"),
                     ("ipv6", "u1", (16,)), ("sec_label", "<u4")])
assert LXC_INFO.itemsize == 32
VERIFY_SMAC, VERIFY_DMAC, VERIFY_SIP = 1, 2, 4
# NODE_MAC, bpf/node_config.h:51
NODE_MAC = bytes([0xde, 0xad, 0xbe, 0xef, 0xc0, 0xde])
# frame path status / verdict values (include/cgpu.h) and the drops it adds
FRAME_NOT_CLASSIFIED = 1
DROP_SNAPLEN = -4096
DROP_INVALID_SMAC, DROP_INVALID_DMAC, DROP_INVALID_SIP = -130, -131, -132
DROP_INVALID, DROP_CT_INVALID_HDR, DROP_UNKNOWN_L3 = -134, -135, -139
DROP_INVALID_EXTHDR = -156
EFAULT_LOAD = -14


def lxc_info(mac: bytes, ipv4_raw: int, ipv6: bytes, verify: int, sec_label: int = 0) -> np.ndarray:
    x = np.zeros((), LXC_INFO)
    x["sec_label"] = sec_label
    x["mac"] = np.frombuffer(bytes(mac), np.uint8)
    x["verify"] = verify
    x["ipv4"] = ipv4_raw
    x["ipv6"] = np.frombuffer(bytes(ipv6), np.uint8)
    return x


def htons(x: int) -> int:
    return socket.htons(x)


def ntohs(x: int) -> int:
    return socket.ntohs(x)


def ip4_be(addr: str | int) -> int:
    """IPv4 address -> u32 whose little-endian memory bytes are network order."""
    if isinstance(addr, str):
        b = socket.inet_aton(addr)
    else:
        b = struct.pack(">I", addr)
    return struct.unpack("<I", b)[0]


def be_to_host4(x):
    """network-order u32 (as stored) -> host integer; works on numpy arrays."""
    if isinstance(x, np.ndarray):
        return x.byteswap()
    return struct.unpack(">I", struct.pack("<I", x))[0]


def policy_key(sec_label: int, dport_host: int, proto: int, egress: int,
               pad_bits: int = 0) -> np.ndarray:
    k = np.zeros((), POLICY_KEY)
    k["sec_label"] = sec_label
    k["dport"] = htons(dport_host)
    k["protocol"] = proto
    k["egress"] = (egress & 1) | (pad_bits << 1)
    return k


def policy_entry(proxy_port_host: int = 0, packets: int = 0, nbytes: int = 0) -> np.ndarray:
    e = np.zeros((), POLICY_ENTRY)
    e["proxy_port"] = htons(proxy_port_host)
    e["packets"] = packets
    e["bytes"] = nbytes
    return e


def ipcache_key(cidr: str, prefixlen_override: int | None = None) -> np.ndarray:
    """pkg/maps/ipcache/ipcache.go:102-123 NewKey."""
    net = ipaddress.ip_network(cidr, strict=False)
    k = np.zeros((), IPCACHE_KEY)
    raw = ipaddress.ip_address(cidr.split("/")[0]).packed
    if net.version == 4:
        k["family"] = ENDPOINT_KEY_IPV4
        k["ip"][:4] = np.frombuffer(raw, np.uint8)
    else:
        k["family"] = ENDPOINT_KEY_IPV6
        k["ip"][:] = np.frombuffer(raw, np.uint8)
    k["prefixlen"] = IPCACHE_STATIC_PREFIX + net.prefixlen if prefixlen_override is None \
        else prefixlen_override
    return k


def remote_info(sec_label: int, tunnel: int = 0) -> np.ndarray:
    v = np.zeros((), REMOTE_ENDPOINT_INFO)
    v["sec_label"] = sec_label
    v["tunnel_endpoint"] = tunnel
    return v


def lpm_key(cidr: str) -> np.ndarray:
    net = ipaddress.ip_network(cidr, strict=False)
    raw = ipaddress.ip_address(cidr.split("/")[0]).packed
    k = np.zeros((), LPM_V4_KEY if net.version == 4 else LPM_V6_KEY)
    k["prefixlen"] = net.prefixlen
    k["addr"][:] = np.frombuffer(raw, np.uint8)
    return k


def endpoint_key(ip: str) -> np.ndarray:
    a = ipaddress.ip_address(ip)
    k = np.zeros((), ENDPOINT_KEY)
    if a.version == 4:
        k["ip"][:4] = np.frombuffer(a.packed, np.uint8)
        k["family"] = ENDPOINT_KEY_IPV4
    else:
        k["ip"][:] = np.frombuffer(a.packed, np.uint8)
        k["family"] = ENDPOINT_KEY_IPV6
    return k


def get_prefix_mask_be(prefix: int) -> int:
    """GET_PREFIX (bpf/lib/ipv6.h:136-138): network-order mask of `prefix` bits."""
    if prefix <= 0:
        h = 0
    elif prefix < 32:
        h = ((1 << prefix) - 1) << (32 - prefix)
    else:
        h = 0xFFFFFFFF
    return ip4_be(h & 0xFFFFFFFF)


def ipv6_addr_clear_suffix(addr16: bytes, prefix: int) -> bytes:
    """ipv6_addr_clear_suffix (bpf/lib/ipv6.h:140-150)."""
    words = list(struct.unpack("<4I", addr16))
    for i in range(4):
        words[i] &= get_prefix_mask_be(prefix)
        prefix -= 32
    return struct.pack("<4I", *words)


def lb4_key(address: str | int, dport_host: int = 0, slave: int = 0) -> np.ndarray:
    """lbmap.NewService4Key(ip, port, slave).ToNetwork() (ipv4.go:99-126)."""
    k = np.zeros((), LB4_KEY)
    k["address"] = ip4_be(address)
    k["dport"] = htons(dport_host)
    k["slave"] = slave
    return k


def lb4_service(target: str | int = 0, port_host: int = 0, count: int = 0, rev_nat: int = 0,
                weight: int = 0) -> np.ndarray:
    """lbmap.NewService4Value(...).ToNetwork() (ipv4.go:144-181)."""
    v = np.zeros((), LB4_SERVICE)
    v["target"] = ip4_be(target)
    v["port"] = htons(port_host)
    v["count"] = count
    v["rev_nat_index"] = htons(rev_nat)
    v["weight"] = htons(weight)
    return v
