"""The closed-form tag-tree rule of k_t2_wave (jp2-bucketeer_amd/csrc/t2_device.hip,
t2_wave_precinct) against the serial walk it replaces (oracle/jp2_oracle.c
tt_set / tt_encode, restated bit for bit below), on random precincts.

k_t2_wave writes every packet header bit in parallel: a code-block's
inclusion-tree bits in packet l come from each node's value v, its parent's
value pv and tp = 1 + the last non-empty packet before l -- no per-node state
-- and its zero-bit-plane bits from the node's first visitor.  The GPU suite
checks whole files; this pins the rule itself, empty packets included.
"""
import random

import pytest


def _levels(w, h):
    out = []
    while True:
        out.append((w, h))
        if w == 1 and h == 1:
            return out
        w, h = (w + 1) >> 1, (h + 1) >> 1


class _Tree:
    """oracle/jp2_oracle.c tt_build / tt_set / tt_encode."""

    def __init__(self, w, h, leaves):
        self.w, self.lv = w, _levels(w, h)
        self.value = [dict() for _ in self.lv]
        for i, v in enumerate(leaves):
            x, y = i % w, i // w
            for k in range(len(self.lv)):
                key = (x >> k, y >> k)
                self.value[k][key] = min(self.value[k].get(key, 1 << 30), v)
        self.low, self.known = {}, {}

    def encode(self, leaf, threshold):
        x, y = leaf % self.w, leaf // self.w
        low, bits = 0, ""
        for k in range(len(self.lv) - 1, -1, -1):
            node = (k, x >> k, y >> k)
            v = self.value[k][(x >> k, y >> k)]
            low = max(low, self.low.get(node, 0))
            while low < threshold:
                if low >= v:
                    if not self.known.get(node):
                        bits += "1"
                        self.known[node] = True
                    break
                bits += "0"
                low += 1
            self.low[node] = low
        return bits


def _serial(w, h, first, zp, L, nonempty):
    """Per packet, per block: the tag-tree bits the serial coder writes."""
    ti, tz = _Tree(w, h, first), _Tree(w, h, zp)
    out = []
    for l in range(L):
        if not nonempty[l]:
            out.append(None)
            continue
        row = []
        for j in range(w * h):
            if first[j] >= l:  # not yet included: the inclusion tree
                b = ti.encode(j, l + 1)
                if first[j] == l:  # included now: the zero bit-plane tree
                    b += tz.encode(j, 1 << 20)
            else:
                b = "-"  # (a plain inclusion bit, not a tag-tree bit)
            row.append(b)
        out.append(row)
    return out


def _closed_form(w, h, first, zp, L, nonempty):
    """The rule t2_wave_precinct applies, lane j = block j."""
    n, nlev = w * h, len(_levels(w, h))
    xy = [(j % w, j // w) for j in range(n)]
    same = [[[(xy[j][0] >> k, xy[j][1] >> k) == (xy[m][0] >> k, xy[m][1] >> k)
              for k in range(nlev)] for j in range(n)] for m in range(n)]
    ival = [[min(first[j] for j in range(n) if same[m][j][k]) for k in range(nlev)] for m in range(n)]
    zval = [[min(zp[j] for j in range(n) if same[m][j][k]) for k in range(nlev)] for m in range(n)]
    zbest = [[min([(first[j] << 6) | j for j in range(n) if same[m][j][k] and first[j] < L], default=1 << 30)
              for k in range(nlev)] for m in range(n)]
    out, tp = [], 0
    for l in range(L):
        if not nonempty[l]:
            out.append(None)
            continue
        vis = [first[j] >= l for j in range(n)]
        row = []
        for m in range(n):
            if not vis[m]:
                row.append("-")
                continue
            b = ""
            for k in range(nlev - 1, -1, -1):
                if any(vis[j] and same[m][j][k] for j in range(m)):
                    continue  # an earlier block visits this node first
                v, pv = ival[m][k], (ival[m][k + 1] if k + 1 < nlev else 0)
                nz = max(0, min(v, l + 1) - max(min(v, tp), min(pv, l + 1)))
                b += "0" * nz + ("1" if tp <= v <= l else "")
            if first[m] == l:
                for k in range(nlev - 1, -1, -1):
                    if zbest[m][k] == ((first[m] << 6) | m):
                        b += "0" * (zval[m][k] - (zval[m][k + 1] if k + 1 < nlev else 0)) + "1"
            row.append(b)
        out.append(row)
        tp = l + 1
    return out


@pytest.mark.parametrize("seed", range(4))
def test_closed_form_tag_trees_equal_the_serial_walk(seed):
    rng = random.Random(seed)
    for _ in range(400):
        w = rng.randint(1, 9)
        h = rng.randint(1, max(1, 64 // w))
        L = rng.randint(1, 10)
        n = w * h
        first = [rng.choice([rng.randint(0, L), L, 0, L - 1]) for _ in range(n)]
        zp = [rng.randint(0, 12) for _ in range(n)]
        # a packet holding a first inclusion is never empty; others may be
        nonempty = [rng.random() < 0.5 or l in first for l in range(L)]
        assert _closed_form(w, h, first, zp, L, nonempty) == _serial(w, h, first, zp, L, nonempty)
