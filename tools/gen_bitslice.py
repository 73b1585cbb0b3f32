"""Generate the bit-sliced RS(10,4) encode XOR program for the gfx950 kernel.

The RS(10,4) parity rows (upstream reed-solomon-erasure's
`Matrix::vandermonde(14, 10) * inv(top 10 rows)` over GF(2^8)/0x11D, called
from /root/reference/helyim-ec/src/encoder.rs:191,208-209) are a FIXED linear
map over GF(2): 80 input bits (10 data bytes) -> 32 output bits (4 parity
bytes) per byte column. Bit-sliced, every 32-bit register holds one bit index
of 32 byte columns ("plane"), so one v_xor / v_bitop3 advances 32 columns of
that bit at once:

    q[8j+b] = XOR over (i, k) with B[(j,b),(i,k)] = 1 of p[8i+k]
    B[(j,b),(i,k)] = bit b of (M[10+j][i] * 2^k)

The 1224 ones of B are shared with common-subexpression elimination (Paar's
greedy pair merging, randomised restarts, best kept under a 3-input-XOR cost
model: a node of t terms costs ceil((t-1)/2) v_bitop3/v_xor ops) and emitted
as straight-line C++ into helyim_amd/csrc/rs104_bitslice.inc. The program is
verified here by simulation against GF multiplication before it is written.

python tools/gen_bitslice.py [--restarts 40] [--seed 1]
"""
from __future__ import annotations

import argparse
import os
import random
from collections import Counter
from itertools import combinations

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
OUT = os.path.join(ROOT, "helyim_amd", "csrc", "rs104_bitslice.inc")

# ---------------------------------------------------------------------------
# GF(2^8) / 0x11D, generator 2 (galois_8; restated, not imported)
EXP = [0] * 512
LOG = [0] * 256
_x = 1
for _i in range(255):
    EXP[_i] = _x
    LOG[_x] = _i
    _x <<= 1
    if _x & 0x100:
        _x ^= 0x11D
for _i in range(255, 512):
    EXP[_i] = EXP[_i - 255]


def gmul(a: int, b: int) -> int:
    return 0 if a == 0 or b == 0 else EXP[LOG[a] + LOG[b]]


def ginv(a: int) -> int:
    return EXP[255 - LOG[a]]


def gexp(a: int, n: int) -> int:
    if n == 0:
        return 1
    return 0 if a == 0 else EXP[(LOG[a] * n) % 255]


def parity_rows(k: int = 10, m: int = 4) -> list[list[int]]:
    """Rows k..k+m-1 of V * inv(V[0..k]) with V[r][c] = r^c."""
    n = k + m
    V = [[gexp(r, c) for c in range(k)] for r in range(n)]
    A = [row[:] + [1 if i == j else 0 for j in range(k)] for i, row in enumerate(V[:k])]
    for c in range(k):  # Gauss-Jordan
        p = next(r for r in range(c, k) if A[r][c])
        A[c], A[p] = A[p], A[c]
        iv = ginv(A[c][c])
        A[c] = [gmul(v, iv) for v in A[c]]
        for r in range(k):
            if r != c and A[r][c]:
                f = A[r][c]
                A[r] = [a ^ gmul(f, b) for a, b in zip(A[r], A[c])]
    inv = [row[k:] for row in A]
    rows = []
    for r in range(k, n):
        row = []
        for c in range(k):
            acc = 0
            for t in range(k):
                acc ^= gmul(V[r][t], inv[t][c])
            row.append(acc)
        rows.append(row)
    return rows


def bit_matrix(rows: list[list[int]]) -> list[set[int]]:
    """Output plane 8j+b -> set of input planes 8i+k."""
    out = []
    for j, row in enumerate(rows):
        for b in range(8):
            s = set()
            for i, c in enumerate(row):
                for k in range(8):
                    if (gmul(c, 1 << k) >> b) & 1:
                        s.add(8 * i + k)
            out.append(s)
    return out


# ---------------------------------------------------------------------------
def node_cost(nterms: int) -> int:
    return (nterms - 1 + 1) // 2 if nterms > 1 else 0  # ceil((t-1)/2) 3-input XORs


def paar(rows: list[set[int]], nin: int, rng: random.Random, min_use: int):
    """Greedy pair merging with random tie-breaks. Returns (nodes, rows):
    nodes[v] = frozenset of the terms of intermediate v (v >= nin)."""
    rows = [set(r) for r in rows]
    nodes: dict[int, list[int]] = {}
    nxt = nin
    while True:
        cnt = Counter()
        for r in rows:
            for a, b in combinations(sorted(r), 2):
                cnt[(a, b)] += 1
        if not cnt:
            break
        best = max(cnt.values())
        if best < min_use:
            break
        cands = [p for p, n in cnt.items() if n == best]
        a, b = rng.choice(cands)
        for r in rows:
            if a in r and b in r:
                r.discard(a)
                r.discard(b)
                r.add(nxt)
        nodes[nxt] = [a, b]
        nxt += 1
    return nodes, rows


def inline_single_use(nodes: dict[int, list[int]], rows: list[set[int]]):
    """Fold intermediates used exactly once into their user (saves an op when
    the user's term count stays odd-friendly under 3-input XORs)."""
    nodes = {v: list(t) for v, t in nodes.items()}
    rows = [list(r) for r in rows]
    changed = True
    while changed:
        changed = False
        uses = Counter()
        for t in nodes.values():
            uses.update(t)
        for r in rows:
            uses.update(r)
        for v in sorted(nodes):
            if uses[v] != 1:
                continue
            for holder in list(nodes.values()) + rows:
                if v in holder:
                    before = node_cost(len(holder)) + node_cost(len(nodes[v]))
                    after = node_cost(len(holder) - 1 + len(nodes[v]))
                    if after <= before:
                        holder.remove(v)
                        holder.extend(nodes[v])
                        del nodes[v]
                        changed = True
                    break
            if changed:
                break
    return nodes, rows


def total_cost(nodes, rows) -> int:
    return sum(node_cost(len(t)) for t in nodes.values()) + sum(node_cost(len(r)) for r in rows)


def simulate(nodes, rows, nin: int, planes: list[int]) -> list[int]:
    val = dict(enumerate(planes))
    for v in sorted(nodes):
        x = 0
        for t in nodes[v]:
            x ^= val[t]
        val[v] = x
    out = []
    for r in rows:
        x = 0
        for t in r:
            x ^= val[t]
        out.append(x)
    return out


def verify(nodes, rows, prows, trials: int = 64) -> None:
    """Random bytes -> planes -> program -> bytes, against GF multiplication."""
    rng = random.Random(7)
    for _ in range(trials):
        cols = [[rng.randrange(256) for _ in range(10)] for _ in range(32)]  # 32 byte columns
        planes = [sum(((cols[c][i] >> k) & 1) << c for c in range(32)) for i in range(10) for k in range(8)]
        q = simulate(nodes, rows, 80, planes)
        for c in range(32):
            for j in range(4):
                want = 0
                for i in range(10):
                    want ^= gmul(prows[j][i], cols[c][i])
                got = sum(((q[8 * j + b] >> c) & 1) << b for b in range(8))
                assert got == want, (c, j, got, want)


def emit(nodes, rows, prows, cost, path: str) -> None:
    def name(t: int) -> str:
        return f"p[{t}]" if t < 80 else f"t{t}"

    def chain(terms: list[int]) -> str:
        # 3-input groups -> v_bitop3_b32 (xor3, gfx950); a leftover pair -> v_xor
        terms = sorted(terms, key=lambda t: (t < 80, t))
        expr = None
        while terms:
            take = 3 if expr is None else 2
            if expr is None and len(terms) == 2:
                take = 2
            grp, terms = terms[:take], terms[take:]
            args = ([expr] if expr is not None else []) + [name(t) for t in grp]
            expr = f"hec_xor3({', '.join(args)})" if len(args) == 3 else " ^ ".join(args)
        return expr

    # demand-driven order: each output row is preceded by the intermediates it
    # needs that are not yet computed (shorter live ranges than all-first)
    done: set[int] = set()
    body: list[str] = []

    def need(v: int) -> None:
        if v < 80 or v in done:
            return
        for t in nodes[v]:
            need(t)
        done.add(v)
        body.append(f"    const uint32_t t{v} = {chain(nodes[v])};")

    for o, r in enumerate(rows):
        for t in r:
            need(t)
        body.append(f"    q[{o}] = {chain(r)};")

    lines = [
        "// GENERATED by tools/gen_bitslice.py -- do not edit.",
        "// Bit-sliced RS(10,4) encode over GF(2): p[8i+k] = plane k of data shard i,",
        "// q[8j+b] = plane b of parity shard j. Parity rows (SURVEY.md Appendix A):",
    ]
    for j, r in enumerate(prows):
        lines.append("//   row %d: %s" % (10 + j, " ".join("0x%02x" % c for c in r)))
    lines += [
        f"// {len(nodes)} shared intermediates; {cost} three-input XOR ops per 32 byte columns",
        "// (1224 terms before elimination). Verified by simulation in the generator.",
        "// Included by bitslice.hpp (hec_xor3, HEC_DEVICE).",
        "#pragma once",
        "HEC_DEVICE void rs104_encode_planes(const uint32_t (&p)[80], uint32_t (&q)[32]) {",
    ] + body + ["}"]
    with open(path, "w") as f:
        f.write("\n".join(lines) + "\n")


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--restarts", type=int, default=40)
    ap.add_argument("--seed", type=int, default=1)
    ap.add_argument("--out", default=OUT)
    args = ap.parse_args()
    prows = parity_rows()
    assert prows[0] == [0x81, 0x96, 0xAF, 0xB8, 0xD2, 0xC4, 0xFE, 0xE8, 0x03, 0x02], prows[0]
    B = bit_matrix(prows)
    assert sum(len(r) for r in B) == 1224
    rng = random.Random(args.seed)
    best = None
    for it in range(args.restarts):
        nodes, rows = paar(B, 80, rng, min_use=2 if it % 2 == 0 else 3)
        nodes, rows = inline_single_use(nodes, rows)
        c = total_cost(nodes, rows)
        if best is None or c < best[0]:
            best = (c, nodes, rows)
    cost, nodes, rows = best
    # renumber intermediates densely in creation order
    order = sorted(nodes)
    ren = {v: 80 + n for n, v in enumerate(order)}
    f = lambda t: ren.get(t, t)
    nodes = {ren[v]: [f(t) for t in nodes[v]] for v in order}
    rows = [[f(t) for t in r] for r in rows]
    verify(nodes, rows, prows)
    emit(nodes, rows, prows, cost, args.out)
    print(f"intermediates {len(nodes)}, xor3-cost {cost}, written {os.path.relpath(args.out, ROOT)}")


if __name__ == "__main__":
    main()
