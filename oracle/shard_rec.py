"""ORACLE — test infrastructure only.

Restatement of the engine's full-pass record (pe_shard_rec / SweepRec,
nomad_amd/csrc/engine_types.h) over the oracle's traced per-row outcomes, so
the sharded protocol (nomad_amd/shard.py) runs on CPU ranks against the
oracle: LimitIterator with limit >= options returns every option with the
first three non-positive ones moved to the end, MaxScoreIterator takes the
first strict maximum. Same 80-byte layout as the C
struct, so records from either side gather alike.
"""
from __future__ import annotations

import ctypes as C
import struct

import numpy as np

from nomad_amd import abi
from nomad_amd.stack import RankedNode

from .oracle import OracleGenericStack, load

FMT = "<d4I3I4I4x3d"
NONE = 0xFFFFFFFF
MAX_SKIP = 3


def empty():
    return {"max": float("-inf"), "max_rank": [NONE] * 4, "np_rank": [NONE] * 3, "np_score": [0.0] * 3,
            "options": 0, "filtered": 0, "exhausted": 0}


def _ins_rank(lst, x):
    lst.append(x)
    lst.sort()
    del lst[len(lst) - 1:]


def _ins_np(r, rank, score):
    pairs = sorted(list(zip(r["np_rank"], r["np_score"])) + [(rank, score)], key=lambda p: p[0])[:MAX_SKIP]
    r["np_rank"] = [p[0] for p in pairs]
    r["np_score"] = [p[1] for p in pairs]


def add(r, rank, score):
    r["options"] += 1
    if score > r["max"]:
        r["max"] = score
        r["max_rank"] = [rank, NONE, NONE, NONE]
    elif score == r["max"]:
        _ins_rank(r["max_rank"], rank)
    if score <= 0.0:
        _ins_np(r, rank, score)


def merge(a, b):
    if b["max"] > a["max"]:
        a["max"] = b["max"]
        a["max_rank"] = list(b["max_rank"])
    elif b["max"] == a["max"]:
        for x in b["max_rank"]:
            _ins_rank(a["max_rank"], x)
    for x, s in zip(b["np_rank"], b["np_score"]):
        _ins_np(a, x, s)
    for k in ("options", "filtered", "exhausted"):
        a[k] += b[k]
    return a


def winner(r):
    if r["options"] == 0:
        return NONE
    if r["max"] > 0.0:
        return r["max_rank"][0]
    for x in r["max_rank"]:
        if x == NONE:
            break
        if x not in r["np_rank"]:
            return x
    return r["max_rank"][0]


def pack(r) -> bytes:
    return struct.pack(FMT, r["max"], *r["max_rank"], *r["np_rank"], r["options"], r["filtered"],
                       r["exhausted"], 0, *r["np_score"])


def unpack(b: bytes):
    v = struct.unpack(FMT, b)
    return {"max": v[0], "max_rank": list(v[1:5]), "np_rank": list(v[5:8]), "options": v[8],
            "filtered": v[9], "exhausted": v[10], "np_score": list(v[12:15])}


class OracleShardStack(OracleGenericStack):
    """OracleGenericStack with SelectShard / SelectMerge: the shard record is
    built from a traced full pass of the oracle chain (oracle_full_pass)."""

    def SelectShard(self, tg, row_begin, row_end) -> bytes:
        lib = load()
        n = len(self.state.row_of) if hasattr(self.state, "row_of") else len(self.nodes)
        st = np.zeros(n, dtype=np.uint8)
        sc = np.zeros(n, dtype=np.float64)
        out = abi.pe_ranked_node()
        rc = lib.oracle_full_pass(self._h, self._tg_index(tg), st.ctypes.data_as(abi.u8p),
                                  sc.ctypes.data_as(abi.f64p), C.byref(out))
        self._check(rc)
        self._last = (st, sc, out.new_offset)
        visit = self._visit
        pos_of = np.full(n, NONE, dtype=np.int64)
        pos_of[visit] = np.arange(len(visit))
        off = out.new_offset   # a full pass leaves the cursor where it was
        r = empty()
        for row in range(row_begin, row_end):
            if pos_of[row] == NONE or st[row] == 255:
                continue
            if st[row] == 1:
                r["filtered"] += 1
            elif st[row] == 2:
                r["exhausted"] += 1
            else:
                add(r, int((pos_of[row] - off) % len(visit)), float(sc[row]))
        return pack(r)

    def SelectMerge(self, tg, recs) -> RankedNode:
        r = empty()
        for b in recs:
            merge(r, unpack(b))
        st, sc, off = self._last
        rank = winner(r)
        n = len(self._visit)
        if rank == NONE:
            return RankedNode(row=-1, node=None, final_score=0.0, nodes_evaluated=n,
                              nodes_filtered=r["filtered"], nodes_exhausted=r["exhausted"], new_offset=off)
        row = int(self._visit[(off + rank) % n])
        return RankedNode(row=row, node=None, final_score=float(sc[row]), nodes_evaluated=n,
                          nodes_filtered=r["filtered"], nodes_exhausted=r["exhausted"], new_offset=off)
