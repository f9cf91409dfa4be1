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


@dataclass
class IngressRule:
    from_requires: list = field(default_factory=list)
    from_endpoints: list = field(default_factory=list)
    to_ports: bool = False


@dataclass
class EgressRule:
    to_requires: list = field(default_factory=list)
    to_endpoints: list = field(default_factory=list)
    to_ports: bool = False


@dataclass
class Rule:
    endpoint_selector: EndpointSelector
    ingress: list = field(default_factory=list)
    egress: list = field(default_factory=list)


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


class Repository:
    """pkg/policy.Repository, rule order kept (repository.go:80-130)."""

    def __init__(self):
        self.rules: list[Rule] = []

    def add(self, rule: Rule):
        self.rules.append(rule)

    def compile(self, strings: Interner | None = None):
        """-> L3Program: selectors, requirements, values, the subject selector
        of every rule and its clauses in rule order (CSR)."""
        st = strings or Interner()
        sels, reqs, vals = [], [], []
        sel_ids = {}

        def selector(es: EndpointSelector) -> int:
            key = (tuple(sorted(es.match_labels.items())),
                   tuple((k, o, tuple(v)) for k, o, v in es.match_expressions))
            if key in sel_ids:
                return sel_ids[key]
            off = len(reqs)
            for k, op, vs in es.requirements():
                ck_src, _, ck_key = k.partition(PATH_DELIMITER)  # GetCiliumKeyFrom
                if not _:
                    ck_src, ck_key = SOURCE_ANY, ck_src
                anysrc = ck_src == SOURCE_ANY
                kid = st("k:" + ck_key) if anysrc else st("x:" + ck_src + PATH_DELIMITER + ck_key)
                reqs.append((1 if anysrc else 0, kid, op, len(vals), len(vs)))
                vals.extend(st("v:" + v) for v in vs)
            sels.append((off, len(reqs) - off, 1 if es.match_all() else 0))
            sel_ids[key] = len(sels) - 1
            return sel_ids[key]

        subject, clauses, coff = [], [], [0]
        for r in self.rules:
            subject.append(selector(r.endpoint_selector))
            # canReachIngress / canReachEgress (rule.go:323-405)
            for ing in r.ingress:
                for s in ing.from_requires:
                    clauses.append((DIR_INGRESS, KIND_REQUIRES, selector(s), 0))
            for ing in r.ingress:
                for s in ing.from_endpoints:
                    clauses.append((DIR_INGRESS, KIND_ALLOWS, selector(s), 1 if ing.to_ports else 0))
            for eg in r.egress:
                for s in eg.to_requires:
                    clauses.append((DIR_EGRESS, KIND_REQUIRES, selector(s), 0))
            for eg in r.egress:
                for s in eg.to_endpoints:
                    clauses.append((DIR_EGRESS, KIND_ALLOWS, selector(s), 1 if eg.to_ports else 0))
            coff.append(len(clauses))
        return L3Program(np.array(sels, SELECTOR), np.array(reqs, REQUIREMENT),
                         np.array(vals, np.uint32), np.array(subject, np.uint32),
                         np.array(coff, np.uint32), np.array(clauses, CLAUSE), st)


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
