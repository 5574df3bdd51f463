"""Independent pure-Python restatement of the reference STARK v1 prover —
SECOND ORACLE, test infrastructure only (small inputs: T <= a few hundred).

Written directly from the reference sources, deliberately with different
formulations from the C oracle so the two can cross-check each other where no
reference artifact pins the v1 bytes (SURVEY.md §8c "parity unpinned"):
  * NTT/INTT as the reference's naive O(n^2) `dft`/`idft`
    (crates/sezkp-ffts/src/lib.rs:191-224) instead of radix-2;
  * BLAKE3 tree mode via the spec's recursive left-subtree split instead of
    the incremental CV stack;
  * the transcript keeps its whole absorbed byte stream and re-hashes it for
    every challenge (crates/sezkp-crypto/src/lib.rs:92-123).
"""
from __future__ import annotations

import struct

P = 0xFFFFFFFF00000001
M32 = 0xFFFFFFFF

# ------------------------------------------------------------------ BLAKE3
IV = [0x6A09E667, 0xBB67AE85, 0x3C6EF372, 0xA54FF53A, 0x510E527F, 0x9B05688C, 0x1F83D9AB, 0x5BE0CD19]
PERM = [2, 6, 3, 10, 7, 0, 4, 13, 1, 11, 12, 5, 9, 14, 15, 8]
CHUNK_START, CHUNK_END, PARENT, ROOT = 1, 2, 4, 8


def _rotr(x, n):
    return ((x >> n) | (x << (32 - n))) & M32


def _compress(cv, words, counter, blen, flags):
    v = list(cv) + IV[:4] + [counter & M32, (counter >> 32) & M32, blen, flags]
    m = list(words)

    def g(a, b, c, d, x, y):
        v[a] = (v[a] + v[b] + x) & M32
        v[d] = _rotr(v[d] ^ v[a], 16)
        v[c] = (v[c] + v[d]) & M32
        v[b] = _rotr(v[b] ^ v[c], 12)
        v[a] = (v[a] + v[b] + y) & M32
        v[d] = _rotr(v[d] ^ v[a], 8)
        v[c] = (v[c] + v[d]) & M32
        v[b] = _rotr(v[b] ^ v[c], 7)

    for rnd in range(7):
        g(0, 4, 8, 12, m[0], m[1]); g(1, 5, 9, 13, m[2], m[3])
        g(2, 6, 10, 14, m[4], m[5]); g(3, 7, 11, 15, m[6], m[7])
        g(0, 5, 10, 15, m[8], m[9]); g(1, 6, 11, 12, m[10], m[11])
        g(2, 7, 8, 13, m[12], m[13]); g(3, 4, 9, 14, m[14], m[15])
        m = [m[PERM[i]] for i in range(16)]
    return [v[i] ^ v[i + 8] for i in range(8)] + [v[i + 8] ^ cv[i] for i in range(8)]


def _words(block: bytes):
    return list(struct.unpack("<16I", block.ljust(64, b"\0")))


def _chunk_node(data: bytes, counter: int):
    """Returns (cv, last_block_words, counter, blen, flags) = the chunk's output node."""
    cv = IV
    blocks = [data[i:i + 64] for i in range(0, len(data), 64)] or [b""]
    for bi, blk in enumerate(blocks):
        flags = (CHUNK_START if bi == 0 else 0) | (CHUNK_END if bi == len(blocks) - 1 else 0)
        if bi == len(blocks) - 1:
            return (cv, _words(blk), counter, len(blk), flags)
        cv = _compress(cv, _words(blk), counter, 64, flags)[:8]


def _node_cv(node):
    cv, w, ctr, blen, flags = node
    return _compress(cv, w, ctr, blen, flags)[:8]


def _tree_node(data: bytes, chunk0: int):
    if len(data) <= 1024:
        return _chunk_node(data, chunk0)
    chunks = (len(data) + 1023) // 1024
    left = 1
    while left * 2 < chunks:
        left *= 2          # largest power of two chunks, leaving >= 1 byte for the right
    l = _node_cv(_tree_node(data[:left * 1024], chunk0))
    r = _node_cv(_tree_node(data[left * 1024:], chunk0 + left))
    return (IV, l + r, 0, 64, PARENT)


def blake3(data: bytes, out_len: int = 32) -> bytes:
    cv, w, _ctr, blen, flags = _tree_node(bytes(data), 0)
    out = b""
    t = 0
    while len(out) < out_len:
        out += struct.pack("<16I", *_compress(cv, w, t, blen, flags | ROOT))
        t += 1
    return out[:out_len]


# ---------------------------------------------------------------- Transcript
class Transcript:
    """crates/sezkp-crypto/src/lib.rs:74-123 — the BLAKE3 state is the hash of
    everything absorbed so far, so keep the stream and re-hash."""

    def __init__(self, dom: str):
        d = dom.encode()
        self.stream = b"sezkp.transcript.v0" + struct.pack("<I", len(d)) + d

    def absorb(self, label: str, data: bytes):
        lb = label.encode()
        self.stream += b"absorb" + struct.pack("<I", len(lb)) + lb + struct.pack("<I", len(data)) + bytes(data)

    def absorb_u64(self, label: str, x: int):
        self.absorb(label, struct.pack("<Q", x))

    def challenge(self, label: str, n: int) -> bytes:
        lb = label.encode()
        out = blake3(self.stream + b"challenge" + struct.pack("<I", len(lb)) + lb, n)
        self.stream += b"after_challenge" + struct.pack("<I", len(lb)) + lb
        return out


# --------------------------------------------------------------------- field
def inv(a):
    return pow(a, P - 2, P)


def f_i64(x):
    return x % P


def root_2exp(k):
    return pow(7, (P - 1) >> k, P)


def dft(a, omega):  # lib.rs:191-202
    n = len(a)
    return [sum(a[j] * pow(omega, j * k, P) for j in range(n)) % P for k in range(n)]


def idft(y, omega):  # lib.rs:209-224
    n = len(y)
    inv_n, oi = inv(n % P), inv(omega)
    return [sum(y[k] * pow(oi, j * k, P) for k in range(n)) % P * inv_n % P for j in range(n)]


# -------------------------------------------------------------------- Merkle
def h2(a, b):
    return blake3(a + b)


def leaf(v):
    return blake3(struct.pack("<Q", v))


def leaf_lab(v, label):
    lb = label.encode()
    return blake3(b"col_leaf" + struct.pack("<I", len(lb)) + lb + struct.pack("<Q", v))


def tree_levels(leaves):  # merkle.rs:46-71
    lvl = list(leaves) or [b"\0" * 32]
    levels = [lvl]
    while len(lvl) > 1:
        lvl = [h2(lvl[i], lvl[i + 1]) if i + 1 < len(lvl) else lvl[i] for i in range(0, len(lvl), 2)]
        levels.append(lvl)
    return levels


def frontier_root(leaves):  # sezkp-merkle lib.rs:167-208 (Frontier push_leaf / finalize_root)
    slots = []  # slots[l]: pending node at level l, or None
    for h in leaves:
        lvl = 0
        while True:
            if len(slots) <= lvl:
                slots.append(None)
            if slots[lvl] is None:
                slots[lvl] = h
                break
            h, slots[lvl] = h2(slots[lvl], h), None
            lvl += 1
    acc = None
    for node in reversed(slots):  # highest level first: parent(higher, lower)
        if node is not None:
            acc = node if acc is None else h2(acc, node)
    return acc if acc is not None else b"\0" * 32


def tree_open(levels, idx):  # merkle.rs:80-108
    idx %= len(levels[0])
    sibs = []
    for lvl in levels[:-1]:
        s = idx ^ 1 if (idx ^ 1) < len(lvl) else idx
        sibs.append(lvl[s])
        idx >>= 1
    return sibs


# ---------------------------------------------------------------- v1 prover
KINDS = ["mv", "wflag", "wsym", "head", "winlen", "in_off", "out_off"]


def labels(tau):  # openings.rs:89-116
    return ["input_mv", "is_first", "is_last"] + [f"{k}_{r}" for k in KINDS for r in range(tau)]


def row_snapshots(blocks):
    """RowIter (openings.rs:182-273): one dict label->field value per row."""
    tau = len(blocks[0]["windows"]) if blocks else 0
    rows = []
    for b in blocks:
        blen = b["step_hi"] - b["step_lo"] + 1
        heads = [0] * tau
        wl = [abs(b["windows"][r]["right"] - b["windows"][r]["left"]) + 1 for r in range(tau)]
        for j in range(blen):
            st = b["movement_log"]["steps"][j]
            row = {"input_mv": f_i64(st["input_mv"]), "is_first": int(j == 0), "is_last": int(j + 1 == blen)}
            for r in range(tau):
                op = st["tapes"][r]
                heads[r] += op["mv"]
                row[f"mv_{r}"] = f_i64(op["mv"])
                row[f"wflag_{r}"] = int(op["write"] is not None)
                row[f"wsym_{r}"] = (op["write"] or 0) % P
                row[f"head_{r}"] = f_i64(heads[r])
                row[f"winlen_{r}"] = wl[r] % P
                row[f"in_off_{r}"] = b["head_in_offsets"][r] % P
                row[f"out_off_{r}"] = b["head_out_offsets"][r] % P
            rows.append(row)
    return rows, tau


def compose(rows, tau, i, a):  # air.rs:49-136 with alpha reuse (prover.rs:86-98)
    n = len(rows)
    R, R1 = rows[i], rows[(i + 1) % n]
    acc = 0
    for r in range(tau):
        mv, flg, head = R[f"mv_{r}"], R[f"wflag_{r}"], R[f"head_{r}"]
        acc += a[0] * flg * (flg - 1)
        acc += a[1] * mv * (mv - 1) * (mv + 1)
        acc += a[2] * (1 - R["is_last"]) * (R1[f"head_{r}"] - head - R1[f"mv_{r}"])
        hb = [(head >> k) & 1 for k in range(16)]
        acc += a[3] * flg * sum(x * (x - 1) for x in hb)
        acc += a[4] * flg * (head - sum(x << k for k, x in enumerate(hb)))
        slack = (R[f"winlen_{r}"] - 1 - head) % P
        sb = [(slack >> k) & 1 for k in range(16)]
        acc += a[5] * flg * sum(x * (x - 1) for x in sb)
        acc += a[6] * flg * (slack - sum(x << k for k, x in enumerate(sb)))
        sym = R[f"wsym_{r}"]
        yb = [(sym >> k) & 1 for k in range(4)]
        acc += a[7] * flg * sum(x * (x - 1) for x in yb)
        acc += a[0] * flg * (sym - sum(x << k for k, x in enumerate(yb)))
        acc += a[2] * R["is_first"] * (head - mv - R[f"in_off_{r}"])
        acc += a[2] * R["is_last"] * (head - R[f"out_off_{r}"])
    return acc % P


def prove_v1(blocks, manifest_root: bytes) -> bytes:
    rows, tau = row_snapshots(blocks)
    n = len(rows)
    assert n and n & (n - 1) == 0
    labs = labels(tau)
    tr = Transcript("sezkp-stark/v1")
    tr.absorb("manifest_root", manifest_root)
    tr.absorb_u64("n", n)
    tr.absorb_u64("tau", tau)
    # column commitments with 1024-row chunks (openings.rs:306-398)
    chunk_trees, outer_trees = {}, {}
    for lab in labs:
        lv = [leaf_lab(r[lab], lab) for r in rows]
        cts = [tree_levels(lv[s:s + 1024]) for s in range(0, n, 1024)]
        chunk_trees[lab] = cts
        outer_trees[lab] = tree_levels([t[-1][0] for t in cts])
    tr.absorb_u64("n_cols", len(labs))
    for lab in labs:
        tr.absorb("col_root", outer_trees[lab][-1][0])
    ab = tr.challenge("alphas", 64)
    a = [int.from_bytes(ab[8 * i:8 * i + 8], "little") % P for i in range(8)]
    tr.absorb("masks", b"masks")
    tr.absorb_u64("n_masks", 1)
    tr.absorb_u64("deg", 4)
    mask = [int.from_bytes(tr.challenge("mask_coeff", 8), "little") % P for _ in range(4)]
    k0 = n.bit_length() - 1
    k = k0 + 3
    N = 1 << k
    z = int.from_bytes(tr.challenge("ood_point", 8), "little") % P
    while pow(z * inv(3) % P, 1 << k, P) == 1:
        z = (z + 1) % P
    wb = root_2exp(k0)
    base = []
    for i in range(n):
        x = pow(wb, i, P)
        rmask = (mask[0] + mask[1] * x + mask[2] * x * x + mask[3] * x ** 3) % P
        base.append((compose(rows, tau, i, a) + rmask) % P)
    coeffs = idft(base, wb) if n > 1 else list(base)
    wN = root_2exp(k)
    g = [coeffs[j] * pow(3, j, P) % P for j in range(n)] + [0] * (N - n)
    y = dft(g, wN)
    lde = [y[i] * inv((3 * pow(wN, i, P) - z) % P) % P for i in range(N)]
    layers = [lde]
    trees = [tree_levels([leaf(v) for v in lde])]
    roots = [trees[0][-1][0]]
    tr.absorb("fri_layer_root", roots[0])
    bb = tr.challenge("fri_betas", 8 * k)
    betas = [int.from_bytes(bb[8 * i:8 * i + 8], "little") % P for i in range(k)]
    for r in range(k):
        cur = layers[-1]
        h = len(cur) // 2
        nxt = [(cur[i] + betas[r] * cur[i + h]) % P for i in range(h)]
        layers.append(nxt)
        trees.append(tree_levels([leaf(v) for v in nxt]))
        roots.append(trees[-1][-1][0])
        tr.absorb("fri_layer_root", roots[-1])
    qb = tr.challenge("row_queries", 240)
    qrows = [int.from_bytes(qb[8 * i:8 * i + 8], "little") % n for i in range(30)]
    fb = tr.challenge("row_queries", 240)
    frows = [int.from_bytes(fb[8 * i:8 * i + 8], "little") % N for i in range(30)]

    U = lambda x: struct.pack("<Q", x)
    vec32 = lambda xs: U(len(xs)) + b"".join(xs)

    def opening(lab, row):
        ch, ii = row // 1024, row % 1024
        t = chunk_trees[lab][ch]
        return (U(rows[row][lab]) + U(row) + U(ch) + U(ii) + t[-1][0] + vec32(tree_open(t, ii))
                + vec32(tree_open(outer_trees[lab], ch)))

    out = U(N) + U(tau) + U(len(labs))
    for lab in labs:
        out += U(len(lab)) + lab.encode() + outer_trees[lab][-1][0]
    out += U(30)
    for row in qrows:
        ip1 = row + 1 if row + 1 < n else 0
        out += U(row) + U(tau)
        for r in range(tau):
            out += (opening(f"mv_{r}", row) + opening(f"mv_{r}", ip1) + opening(f"wflag_{r}", row)
                    + opening(f"wsym_{r}", row) + opening(f"head_{r}", row) + opening(f"head_{r}", ip1)
                    + opening(f"winlen_{r}", row) + opening(f"in_off_{r}", row) + opening(f"out_off_{r}", row))
        out += opening("is_first", row) + opening("is_last", row) + opening("input_mv", row)
    out += vec32(roots) + U(30)
    for idx0 in frows:
        pos = [idx0]
        ln = N
        for r in range(k):
            pos.append(pos[-1] % (ln // 2))
            ln //= 2
        out += U(len(pos)) + b"".join(U(p) for p in pos) + U(k)
        ln = N
        for r in range(k):
            i, j = pos[r], pos[r] ^ (ln // 2)
            out += (U(layers[r][i]) + vec32(tree_open(trees[r], i)) + U(layers[r][j])
                    + vec32(tree_open(trees[r], j)))
            ln //= 2
    out += U(layers[k][0]) + bytes(manifest_root)
    return out
