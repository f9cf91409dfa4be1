"""L3 MapState compilation: the label side of the policy
repository, compiled into integer tables for the batched selector match of
cgpu_l3_compile.

Mirrors, for the L3 (label-only) decision that computeDesiredL3PolicyMapEntries
(pkg/endpoint/policy.go:317-390) asks of the repository:

* labels      pkg/labels/labels.go:405-417 (GetExtendedKey, GetCiliumKeyFrom),
              :579-637 (parseSource, ParseLabel, ParseSelectLabel)
* LabelArray  pkg/labels/array.go:92-130 (Has / Get with the "any" source)
* selectors   pkg/policy/api/selector.go:177-302 (NewESFromLabels,
              NewESFromMatchRequirements, Matches with "reserved.all") over
              k8s.io/apimachinery labels.Requirement.Matches (In / NotIn /
              Exists / DoesNotExist)
* rules       pkg/policy/rule.go:323-405 (canReachIngress / canReachEgress:
              FromRequires/ToRequires first, then FromEndpoints/ToEndpoints
              without ToPorts), pkg/policy/repository.go:80-130, :443-490
              (CanReach*RLocked: a Denied rule ends the walk as Denied, an
              Allowed one is kept; Allows*LabelAccess: Allowed only if the
              walk ended Allowed)

Strings are interned on the host; the device sees ids only.  The restatement
in oracle/cgpu_oracle.c (or_l3_compile) reads the same tables.
"""
from __future__ import annotations

import ctypes as C
from dataclasses import dataclass, field

import numpy as np

PATH_DELIMITER = "."
SOURCE_ANY = "any"
SOURCE_UNSPEC = "unspec"
SOURCE_RESERVED = "reserved"

OP_IN, OP_NOT_IN, OP_EXISTS, OP_NOT_EXISTS = 0, 1, 2, 3
_OPS = {"In": OP_IN, "=": OP_IN, "==": OP_IN, "NotIn": OP_NOT_IN, "!=": OP_NOT_IN,
        "Exists": OP_EXISTS, "DoesNotExist": OP_NOT_EXISTS}
DIR_INGRESS, DIR_EGRESS = 0, 1
KIND_REQUIRES, KIND_ALLOWS = 0, 1
L3_INGRESS_ENFORCED, L3_EGRESS_ENFORCED = 1, 2


@dataclass(frozen=True)
class Label:
    source: str
    key: str
    value: str = ""

    def extended_key(self) -> str:  # labels.go:405-407
        return self.source + PATH_DELIMITER + self.key


def _parse_source(s: str):  # labels.go:579-600
    if s == "":
        return "", ""
    if s[0] == "$":
        s = s.replace("$", SOURCE_RESERVED + ":", 1)
    parts = s.split(":", 1)
    src = ""
    if len(parts) != 2:
        nxt = parts[0]
        if nxt.startswith(SOURCE_RESERVED):
            src = SOURCE_RESERVED
            nxt = nxt[len(SOURCE_RESERVED + PATH_DELIMITER):] if nxt.startswith(
                SOURCE_RESERVED + PATH_DELIMITER) else nxt
    else:
        if parts[0] != "":
            src = parts[0]
        nxt = parts[1]
    return src, nxt


def parse_label(s: str) -> Label:  # labels.go:605-624
    src, nxt = _parse_source(s)
    source = src if src != "" else SOURCE_UNSPEC
    kv = nxt.split("=", 1)
    key, value = kv[0], ""
    if len(kv) > 1:
        if src == SOURCE_RESERVED and kv[0] == "":
            key = kv[1]
        else:
            value = kv[1]
    return Label(source, key, value)


def parse_select_label(s: str) -> Label:  # labels.go:629-637
    lbl = parse_label(s)
    if lbl.source == SOURCE_UNSPEC:
        lbl = Label(SOURCE_ANY, lbl.key, lbl.value)
    return lbl


def parse_select_label_array(*ss: str):
    return [parse_select_label(s) for s in ss]


def parse_label_array(*ss: str):
    return [parse_label(s) for s in ss]


@dataclass
class EndpointSelector:
    """matchLabels {extended key: value} + matchExpressions [(key, op, values)]."""
    match_labels: dict = field(default_factory=dict)
    match_expressions: list = field(default_factory=list)

    @staticmethod
    def from_labels(*labels: Label) -> "EndpointSelector":  # selector.go:177-185
        return EndpointSelector({l.extended_key(): l.value for l in labels})

    def requirements(self):
        """metav1.LabelSelectorAsSelector: one In requirement per matchLabels
        entry, then the expressions (order does not change the result)."""
        reqs = [(k, OP_IN, (v,)) for k, v in sorted(self.match_labels.items())]
        for k, op, vals in self.match_expressions:
            reqs.append((k, _OPS[op] if isinstance(op, str) else op, tuple(vals)))
        return reqs

    def match_all(self) -> bool:  # selector.go:290-294
        return (SOURCE_RESERVED + PATH_DELIMITER + "all") in self.match_labels


WILDCARD = EndpointSelector()  # api.WildcardEndpointSelector = NewESFromLabels() (selector.go:223)


def is_wildcard(es: EndpointSelector) -> bool:  # selector.go:305-308
    return not es.match_labels and not es.match_expressions


def selects_all(sels) -> bool:  # EndpointSelectorSlice.SelectsAllEndpoints (selector.go:356-368)
    return len(sels) == 0 or any(is_wildcard(s) for s in sels)


def reserved_selector(name: str) -> EndpointSelector:  # newReservedEndpointSelector (selector.go:215-218)
    return EndpointSelector.from_labels(Label(SOURCE_RESERVED, name, ""))


# api.EntitySelectorMapping (pkg/policy/api/entity.go:47-69)
ENTITY_SELECTORS = {"all": WILDCARD, "world": reserved_selector("world"),
                    "cluster": reserved_selector("cluster"), "host": reserved_selector("host"),
                    "init": reserved_selector("init")}


def entity_selectors(entities):  # EntitySlice.GetAsEndpointSelectors (entity.go:96-105)
    return [ENTITY_SELECTORS[e] for e in entities if e in ENTITY_SELECTORS]


# ------------------------------------------------------------- CIDR labels
def masked_ip_to_label_string(ip, prefix: int) -> str:
    """labels.maskedIPToLabelString (pkg/labels/cidr.go:28-46): ':' -> '-',
    a leading / trailing '-' padded with '0'."""
    s = str(ip).replace(":", "-")
    if s[0] == "-":
        s = "0" + s
    if s[-1] == "-":
        s = s + "0"
    return f"cidr:{s}/{prefix}"


def _parse_cidr(s: str):
    """net.ParseCIDR (the address masked to the prefix) or, for a bare
    address, a full-length prefix (labels.IPStringToLabel, cidr.go:58-74)."""
    import ipaddress
    try:
        return ipaddress.ip_network(s, strict=False)
    except ValueError:
        pass
    try:
        ip = ipaddress.ip_address(s)
    except ValueError:
        return None
    return ipaddress.ip_network((ip, ip.max_prefixlen))


def ip_string_to_label(s: str):  # labels.IPStringToLabel -> IPNetToLabel (cidr.go:49-74)
    net = _parse_cidr(s)
    if net is None:
        return None
    return parse_label(masked_ip_to_label_string(net.network_address, net.prefixlen))


def cidr_identity_labels(cidr: str, cluster_cidr: str):
    """labels/cidr.GetCIDRLabels (pkg/labels/cidr/cidr.go:33-66): the labels
    of a CIDR identity: the prefix and every shorter one down to /0 (none for
    a /0 itself), then reserved:cluster if the cluster range holds it, else
    reserved:world."""
    import ipaddress
    net = _parse_cidr(cidr)
    ones = net.prefixlen
    out = []
    if ones > 0:
        for i in range(ones + 1):
            sub = net.supernet(new_prefix=i)
            out.append(parse_label(masked_ip_to_label_string(sub.network_address, i)))
    cl = ipaddress.ip_network(cluster_cidr, strict=False)
    inside = (cl.version == net.version and net.network_address in cl and cl.prefixlen <= ones)
    out.append(parse_label("reserved:" + ("cluster" if inside else "world")))
    return out


CIDR_MATCH_ALL = ("0.0.0.0/0", "::/0")  # api.CIDRMatchAll


def cidr_selectors(cidrs):
    """CIDRSlice.GetAsEndpointSelectors (pkg/policy/api/cidr.go:70-86): the
    first match-all CIDR also adds the reserved:world selector."""
    out, world = [], False
    for c in cidrs:
        if c in CIDR_MATCH_ALL and not world:
            world = True
            out.append(reserved_selector("world"))
        lbl = ip_string_to_label(c)
        if lbl is not None:
            out.append(EndpointSelector.from_labels(lbl))
    return out


def _net_key(n):
    return (n[1], n[0].packed)


def remove_cidrs(allow, remove):
    """ip.RemoveCIDRs (pkg/ip/ip.go:124-177) over (address, prefixlen) pairs,
    in the reference's output order; None where it returns an error (mixed
    families, or a remove prefix not strictly inside the allow prefix that
    holds its first address, removeCIDR :194-250)."""
    import ipaddress

    def net(n):
        return ipaddress.ip_network((n[0], n[1]), strict=False)

    remove = sorted(remove, key=_net_key)  # NetsByMask (ip.go:58-74)
    again = True
    while again:  # PreLoop: drop removes that another remove contains
        again = False
        for j, rj in enumerate(remove):
            for i, ri in enumerate(remove):
                if i != j and ri[0].version == rj[0].version and ri[0] in net(rj):
                    del remove[i]
                    again = True
                    break
            if again:
                break
    allow = list(allow)
    for rm in remove:
        rnet = net(rm)
        again = True
        while again:
            again = False
            for i, a in enumerate(allow):
                if a[0].version != rm[0].version:
                    return None
                anet = net(a)
                if rnet.network_address in anet:
                    if a[1] >= rm[1]:
                        return None
                    bits = rnet.max_prefixlen
                    split = []
                    for L in range(a[1] + 1, rm[1] + 1):  # i = bits-a-1 .. bits-r
                        flip = int(rnet.network_address) ^ (1 << (bits - L))
                        flip |= int(anet.network_address)
                        sub = ipaddress.ip_network((flip, L), strict=False) if rnet.version == 6 \
                            else ipaddress.ip_network((ipaddress.IPv4Address(flip & 0xFFFFFFFF), L),
                                                      strict=False)
                        split.append((sub.network_address, L))
                    allow = allow[:i] + allow[i + 1:] + split
                    again = True
                    break
                if anet.network_address in rnet:
                    allow = allow[:i] + allow[i + 1:]
                    again = True
                    break
    return allow


def resultant_cidr_set(cidr_rules):
    """api.ComputeResultantCIDRSet (pkg/policy/api/cidr.go:115-132):
    [(cidr, [except...])] -> CIDR strings; a rule whose RemoveCIDRs fails
    contributes nothing (the error is dropped)."""
    out = []
    for cidr, excepts in cidr_rules:
        a = _parse_cidr(cidr)
        rm = [_parse_cidr(x) for x in excepts]
        res = remove_cidrs([(a.network_address, a.prefixlen)],
                           [(r.network_address, r.prefixlen) for r in rm])
        for ip, L in res or []:
            out.append(f"{ip}/{L}")
    return out


# ------------------------------------------------------------- rules
PROTO_TCP, PROTO_UDP, PROTO_ANY = "TCP", "UDP", "ANY"
U8PROTO = {PROTO_TCP: 6, PROTO_UDP: 17, PROTO_ANY: 0}  # u8proto.ParseProtocol
PARSER_NONE, PARSER_HTTP, PARSER_KAFKA = "", "http", "kafka"


@dataclass
class PortRule:
    """api.PortRule: ports [(port string, "TCP"|"UDP"|"ANY")] and optional L7
    rules (only their presence and kind matter to the MapState)."""
    ports: list = field(default_factory=list)
    http: list = field(default_factory=list)
    kafka: list = field(default_factory=list)

    def rules_empty(self) -> bool:  # L7Rules.IsEmpty
        return not self.http and not self.kafka


class _PeerRule:
    def port_rules(self):
        return self.to_ports if isinstance(self.to_ports, list) else []

    def has_ports(self) -> bool:
        return bool(self.to_ports)


@dataclass
class IngressRule(_PeerRule):
    """api.IngressRule; to_ports is a list of PortRule (a bare True keeps
    the L3 meaning "restricted to some ports" without listing them)."""
    from_requires: list = field(default_factory=list)
    from_endpoints: list = field(default_factory=list)
    to_ports: object = False
    from_entities: list = field(default_factory=list)
    from_cidr: list = field(default_factory=list)
    from_cidr_set: list = field(default_factory=list)

    requires = property(lambda self: self.from_requires)
    endpoints = property(lambda self: self.from_endpoints)

    def peer_selectors(self, endpoints=None):
        """GetSourceEndpointSelectors (pkg/policy/api/ingress.go:111-115)"""
        eps = self.from_endpoints if endpoints is None else endpoints
        return (list(eps) + entity_selectors(self.from_entities) + cidr_selectors(self.from_cidr)
                + cidr_selectors(resultant_cidr_set(self.from_cidr_set)))

    def is_label_based(self) -> bool:  # ingress.go:120-122
        return len(self.from_requires) + len(self.from_cidr) + len(self.from_cidr_set) == 0


@dataclass
class EgressRule(_PeerRule):
    to_requires: list = field(default_factory=list)
    to_endpoints: list = field(default_factory=list)
    to_ports: object = False
    to_entities: list = field(default_factory=list)
    to_cidr: list = field(default_factory=list)
    to_cidr_set: list = field(default_factory=list)
    to_services: int = 0

    requires = property(lambda self: self.to_requires)
    endpoints = property(lambda self: self.to_endpoints)

    def peer_selectors(self, endpoints=None):
        """GetDestinationEndpointSelectors (pkg/policy/api/egress.go:139-143)"""
        eps = self.to_endpoints if endpoints is None else endpoints
        return (list(eps) + entity_selectors(self.to_entities) + cidr_selectors(self.to_cidr)
                + cidr_selectors(resultant_cidr_set(self.to_cidr_set)))

    def is_label_based(self) -> bool:  # egress.go:148-150
        return len(self.to_requires) + len(self.to_cidr) + len(self.to_cidr_set) + self.to_services == 0


@dataclass
class Rule:
    endpoint_selector: EndpointSelector
    ingress: list = field(default_factory=list)
    egress: list = field(default_factory=list)
    labels: list = field(default_factory=list)


def selector_matches(es: EndpointSelector, labels) -> bool:
    """EndpointSelector.Matches (selector.go:277-302) on the host: the same
    rules the device's l3_match applies to interned ids."""
    if es.match_all():
        return True
    for k, op, vals in es.requirements():
        src, dot, key = k.partition(PATH_DELIMITER)
        if not dot:
            src, key = SOURCE_ANY, src
        hit = None
        for l in labels:  # LabelArray.Has / Get (array.go:92-130): first match
            if (l.key == key) if src == SOURCE_ANY else (l.extended_key() == src + PATH_DELIMITER + key):
                hit = l.value
                break
        has = hit is not None
        inn = has and hit in vals
        ok = (has and inn) if op == OP_IN else (not inn) if op == OP_NOT_IN else \
            has if op == OP_EXISTS else not has
        if not ok:
            return False
    return True


def _parse_port(s: str) -> int:
    """strconv.ParseUint(s, 0, 16) with the error ignored (l4.go:156): 0x/0o/0b
    prefixes, a leading 0 means octal; anything invalid or > 65535 is 0."""
    t = s.replace("_", "")
    try:
        if t[:2].lower() in ("0x", "0o", "0b"):
            v = int(t, 0)
        elif len(t) > 1 and t[0] == "0":
            v = int(t[1:], 8)
        else:
            v = int(t, 10)
    except ValueError:
        return 0
    return v if 0 <= v <= 0xFFFF else 0


class PolicyError(Exception):
    """The merge errors of mergeL4{Ingress,Egress}Port (rule.go:75-81)."""


@dataclass
class L4Filter:
    """pkg/policy/l4.go:83-103, the fields the MapState reads."""
    port: int
    protocol: str
    u8proto: int
    endpoints: list
    parser: str
    ingress: bool

    def allows_all(self) -> bool:  # AllowsAllAtL3 (l4.go:106-108)
        return selects_all(self.endpoints)

    def is_redirect(self) -> bool:  # l4.go:222-224
        return self.parser != PARSER_NONE


def _create_l4_filter(peers, pr: PortRule, port: str, proto: str, ingress: bool) -> L4Filter:
    """CreateL4Filter (l4.go:152-186)"""
    eps = [WILDCARD] if selects_all(peers) else list(peers)
    parser = PARSER_NONE
    if proto == PROTO_TCP and not pr.rules_empty():
        parser = PARSER_HTTP if pr.http else PARSER_KAFKA
    return L4Filter(_parse_port(port), proto, U8PROTO[proto], eps, parser, ingress)


def _requirement_selector(es: EndpointSelector, reqs) -> EndpointSelector:
    """FromEndpoints[i].MatchExpressions += requirements (rule.go:218-228)"""
    return EndpointSelector(dict(es.match_labels), list(es.match_expressions) + list(reqs))


def _convert_requirements(es: EndpointSelector):
    """ConvertToLabelSelectorRequirementSlice (selector.go:313-327)"""
    return list(es.match_expressions) + [(k, "In", [v]) for k, v in es.match_labels.items()]


class Interner:
    def __init__(self):
        self.ids = {}

    def __call__(self, s: str) -> int:
        return self.ids.setdefault(s, len(self.ids))


LABEL = np.dtype([("key", "<u4"), ("ext_key", "<u4"), ("value", "<u4")])
REQUIREMENT = np.dtype([("any_source", "<u4"), ("key", "<u4"), ("op", "<u4"),
                        ("values_off", "<u4"), ("n_values", "<u4")])
SELECTOR = np.dtype([("reqs_off", "<u4"), ("n_reqs", "<u4"), ("match_all", "<u4")])
CLAUSE = np.dtype([("dir", "<u4"), ("kind", "<u4"), ("selector", "<u4"), ("has_ports", "<u4")])


class SelectorTable:
    """Interned EndpointSelectors -> (SELECTOR, REQUIREMENT, values) arrays."""

    def __init__(self, strings: Interner):
        self.st = strings
        self.sels, self.reqs, self.vals, self.ids = [], [], [], {}

    def __call__(self, es: EndpointSelector) -> int:
        key = (tuple(sorted(es.match_labels.items())),
               tuple((k, o, tuple(v)) for k, o, v in es.match_expressions))
        if key in self.ids:
            return self.ids[key]
        st, off = self.st, len(self.reqs)
        for k, op, vs in es.requirements():
            ck_src, dot, ck_key = k.partition(PATH_DELIMITER)  # GetCiliumKeyFrom
            if not dot:
                ck_src, ck_key = SOURCE_ANY, ck_src
            anysrc = ck_src == SOURCE_ANY
            kid = st("k:" + ck_key) if anysrc else st("x:" + ck_src + PATH_DELIMITER + ck_key)
            self.reqs.append((1 if anysrc else 0, kid, op, len(self.vals), len(vs)))
            self.vals.extend(st("v:" + v) for v in vs)
        self.sels.append((off, len(self.reqs) - off, 1 if es.match_all() else 0))
        self.ids[key] = len(self.sels) - 1
        return self.ids[key]


class Repository:
    """pkg/policy.Repository, rule order kept (repository.go:80-130)."""

    def __init__(self):
        self.rules: list[Rule] = []

    def add(self, rule: Rule):
        self.rules.append(rule)

    def compile(self, strings: Interner | None = None, table: SelectorTable | None = None):
        """-> L3Program: selectors, requirements, values, the subject selector
        of every rule and its clauses in rule order (CSR).  `table` may
        already hold other selectors (the L4 filters of compile_mapstate)."""
        st = strings or (table.st if table else Interner())
        selector = table or SelectorTable(st)
        subject, clauses, coff = [], [], [0]
        for r in self.rules:
            subject.append(selector(r.endpoint_selector))
            # canReachIngress / canReachEgress (rule.go:323-405): Requires
            # first, then GetSource/DestinationEndpointSelectors
            for d, blocks in ((DIR_INGRESS, r.ingress), (DIR_EGRESS, r.egress)):
                for b in blocks:
                    for s in b.requires:
                        clauses.append((d, KIND_REQUIRES, selector(s), 0))
                for b in blocks:
                    for s in b.peer_selectors():
                        clauses.append((d, KIND_ALLOWS, selector(s), 1 if b.has_ports() else 0))
            coff.append(len(clauses))
        return L3Program(np.array(selector.sels, SELECTOR).reshape(-1),
                         np.array(selector.reqs, REQUIREMENT).reshape(-1),
                         np.array(selector.vals, np.uint32), np.array(subject, np.uint32),
                         np.array(coff, np.uint32), np.array(clauses, CLAUSE).reshape(-1), st)

    # ---------------------------------------------------------------- L4
    def resolve_l4(self, ctx_labels, ingress: bool, wildcard: bool = True) -> dict:
        """ResolveL4IngressPolicy / ResolveL4EgressPolicy (repository.go:240-329)
        -> {"port/PROTO": L4Filter} in insertion order.  ctx_labels is ctx.To
        (ingress) or ctx.From (egress): the endpoint's labels.  wildcard=False
        stops before the wildcardL3L4Rules pass (what the per-rule
        resolveL4*Policy returns)."""
        subj = [selector_matches(r.endpoint_selector, ctx_labels) for r in self.rules]
        reqs = []
        for r, s in zip(self.rules, subj):
            for b in (r.ingress if ingress else r.egress):
                if s:
                    for q in b.requires:
                        reqs.extend(_convert_requirements(q))
        res = {}
        for r, s in zip(self.rules, subj):  # rule.resolveL4{Ingress,Egress}Policy (rule.go:198-244,539-585)
            if not s:
                continue
            for b in (r.ingress if ingress else r.egress):
                eps = [_requirement_selector(e, reqs) for e in b.endpoints] if reqs else b.endpoints
                if not b.has_ports():  # mergeL4{Ingress,Egress} (rule.go:123-186, 413-455)
                    continue
                peers = b.peer_selectors(eps)
                for pr in b.port_rules():
                    for port, proto in pr.ports:
                        for pt in ((proto,) if proto != PROTO_ANY else (PROTO_TCP, PROTO_UDP)):
                            _merge_l4_port(res, peers, pr, port, pt, ingress)
        if wildcard:
            self._wildcard_l3l4(ctx_labels, ingress, res, subj)
        return res

    def _wildcard_l3l4(self, ctx_labels, ingress, res, subj):
        """wildcardL3L4Rules (repository.go:128-230): label-based peers of
        L3-only rules (TCP and UDP, any port) and of L3/L4 rules without L7
        rules (their port, their protocol string: ANY matches no filter) join
        every filter that has an L7 parser."""
        def wl(proto, port, peers):
            for f in res.values():
                if proto != f.protocol or (port != 0 and port != f.port) or f.parser == PARSER_NONE:
                    continue
                f.endpoints = f.endpoints + list(peers)

        for r, s in zip(self.rules, subj):
            if not s:
                continue
            for b in (r.ingress if ingress else r.egress):
                if not b.is_label_based():
                    continue
                peers = b.peer_selectors()
                if not b.has_ports():
                    wl(PROTO_TCP, 0, peers)
                    wl(PROTO_UDP, 0, peers)
                    continue
                for pr in b.port_rules():
                    if pr.rules_empty():
                        for port, proto in pr.ports:
                            wl(proto, _parse_port(port), peers)


def _merge_l4_port(res, peers, pr, port, proto, ingress):
    """mergeL4IngressPort / mergeL4EgressPort (rule.go:46-121, 462-537)"""
    key = port + "/" + proto
    f = _create_l4_filter(peers, pr, port, proto, ingress)
    ex = res.get(key)
    if ex is None:
        res[key] = f
        return
    if ex.allows_all() or f.allows_all():
        ex.endpoints = [WILDCARD]
    else:
        ex.endpoints = ex.endpoints + list(peers)
    if f.parser != PARSER_NONE:
        if ex.parser == PARSER_NONE:
            ex.parser = f.parser
        elif f.parser != ex.parser:
            raise PolicyError(f"Cannot merge conflicting L7 parsers ({f.parser}/{ex.parser})")


@dataclass
class L3Program:
    selectors: np.ndarray
    reqs: np.ndarray
    values: np.ndarray
    rule_subject: np.ndarray
    rule_clauses: np.ndarray  # CSR offsets, n_rules + 1
    clauses: np.ndarray
    strings: Interner

    def label_sets(self, sets):
        """[[Label]] -> (offsets u32[n+1], LABEL records) in array order."""
        st = self.strings
        recs, offs = [], [0]
        for labels in sets:
            for l in labels:
                recs.append((st("k:" + l.key), st("x:" + l.extended_key()), st("v:" + l.value)))
            offs.append(len(recs))
        return np.array(offs, np.uint32), np.array(recs, LABEL)


class CL3Program(C.Structure):
    _fields_ = [("selectors", C.c_void_p), ("n_selectors", C.c_uint32),
                ("reqs", C.c_void_p), ("n_reqs", C.c_uint32),
                ("values", C.c_void_p), ("n_values", C.c_uint32),
                ("rule_subject", C.c_void_p), ("rule_clauses", C.c_void_p), ("n_rules", C.c_uint32),
                ("clauses", C.c_void_p), ("n_clauses", C.c_uint32)]


class CLabelSets(C.Structure):
    _fields_ = [("offsets", C.c_void_p), ("labels", C.c_void_p), ("n_sets", C.c_uint32)]


def c_program(p: L3Program):
    """ctypes view of a program (keep `p` alive while it is used)."""
    def ptr(a):
        return a.ctypes.data if len(a) else None
    return CL3Program(ptr(p.selectors), len(p.selectors), ptr(p.reqs), len(p.reqs),
                      ptr(p.values), len(p.values), ptr(p.rule_subject), p.rule_clauses.ctypes.data,
                      len(p.rule_subject), ptr(p.clauses), len(p.clauses))


def c_label_sets(offs, recs):
    return CLabelSets(offs.ctypes.data, recs.ctypes.data if len(recs) else None, len(offs) - 1)


def desired_l3_keys(allow_row: np.ndarray, identities, flags: int = 3):
    """computeDesiredL3PolicyMapEntries (policy.go:317-390): the PolicyKey
    {identity, 0, 0, direction} of every identity the row allows."""
    from . import layouts as L
    keys = []
    for ident, a in zip(identities, allow_row):
        if a & 1:  # policymap.Ingress = 0
            keys.append(L.policy_key(int(ident), 0, 0, 0))
        if a & 2:  # policymap.Egress = 1
            keys.append(L.policy_key(int(ident), 0, 0, 1))
    return keys


# --------------------------------------------------------- full MapState
L4_FILTER = np.dtype([("endpoint", "<u4"), ("sels_off", "<u4"), ("n_sels", "<u4"), ("port", "<u2"),
                      ("proto", "u1"), ("dir", "u1"), ("proxy_port", "<u2"), ("redirect", "u1"),
                      ("pad", "u1")])
assert L4_FILTER.itemsize == 20
MS_ALLOW_LOCALHOST, MS_HOST_ALLOWS_WORLD = 4, 8
HOST_ID, WORLD_ID = 1, 2


@dataclass
class EndpointPolicy:
    """What computeDesiredPolicyMapState reads of an endpoint: its identity's
    labels, the index of its policy map (the `ep` of cgpu_policy_update), the
    ingress/egressPolicyEnabled flags and realizedRedirects, keyed here by
    (ingress, "TCP"|"UDP", port) instead of the ProxyID string."""
    labels: list
    index: int
    ingress_enforced: bool = True
    egress_enforced: bool = True
    redirects: dict = field(default_factory=dict)


@dataclass
class MapStateProgram:
    prog: L3Program
    ep_sets: tuple
    id_sets: tuple
    filters: np.ndarray
    filter_sels: np.ndarray
    ep_map: np.ndarray
    ep_flags: np.ndarray
    identity: np.ndarray
    l4: list  # per endpoint row: (ingress L4PolicyMap, egress L4PolicyMap)


def compile_mapstate(repo: Repository, endpoints, identities, always_allow_localhost=False,
                     host_allows_world=False) -> MapStateProgram:
    """Everything cgpu_mapstate_sync needs for Endpoint.regeneratePolicy of
    every endpoint: resolveL4Policy (pkg/endpoint/policy.go:222-271) per
    endpoint on the host, its filters' selectors interned next to the rule
    program, and the per-endpoint flags of determineAllowLocalhost /
    determineAllowFromWorld (:284-315).  identities: [(NumericIdentity,
    [Label])] (the identity cache).  Raises PolicyError where
    ResolveL4*Policy returns an error."""
    st = Interner()
    table = SelectorTable(st)
    filters, fsels, flags, l4 = [], [], [], []
    for row, ep in enumerate(endpoints):
        maps = []
        for ingress, enforced in ((True, ep.ingress_enforced), (False, ep.egress_enforced)):
            m = repo.resolve_l4(ep.labels, ingress) if enforced else {}
            maps.append(m)
            for f in m.values():
                off = len(fsels)
                fsels.extend(table(s) for s in f.endpoints)
                proxy = ep.redirects.get((ingress, f.protocol, f.port), 0) if f.is_redirect() else 0
                filters.append((row, off, len(fsels) - off, f.port, f.u8proto,
                                DIR_INGRESS if ingress else DIR_EGRESS, proxy,
                                1 if f.is_redirect() else 0, 0))
        has_redirect = any(f.is_redirect() for m in maps for f in m.values())
        fl = (L3_INGRESS_ENFORCED if ep.ingress_enforced else 0) | \
             (L3_EGRESS_ENFORCED if ep.egress_enforced else 0)
        if always_allow_localhost or has_redirect:
            fl |= MS_ALLOW_LOCALHOST
        if host_allows_world:
            fl |= MS_HOST_ALLOWS_WORLD
        flags.append(fl)
        l4.append(tuple(maps))
    prog = repo.compile(st, table)
    return MapStateProgram(prog, prog.label_sets([e.labels for e in endpoints]),
                           prog.label_sets([lb for _, lb in identities]),
                           np.array(filters, L4_FILTER).reshape(-1), np.array(fsels, np.uint32),
                           np.array([e.index for e in endpoints], np.uint32),
                           np.array(flags, np.uint32),
                           np.array([i for i, _ in identities], np.uint32), l4)


class CMapStateSpec(C.Structure):
    _fields_ = [("filters", C.c_void_p), ("n_filters", C.c_uint32),
                ("filter_sels", C.c_void_p), ("n_filter_sels", C.c_uint32),
                ("ep_map", C.c_void_p), ("ep_flags", C.c_void_p), ("identity", C.c_void_p)]


class CMapStateStats(C.Structure):
    _fields_ = [(n, C.c_uint64) for n in ("desired", "added", "updated", "deleted", "unchanged",
                                          "failed")]


def c_mapstate_spec(m: MapStateProgram):
    def ptr(a):
        return a.ctypes.data if len(a) else None
    return CMapStateSpec(ptr(m.filters), len(m.filters), ptr(m.filter_sels), len(m.filter_sels),
                         ptr(m.ep_map), ptr(m.ep_flags), ptr(m.identity))
