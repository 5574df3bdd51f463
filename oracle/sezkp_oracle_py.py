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
        blen = (b["step_hi"] - b["step_lo"] + 1) % (1 << 64)  # usize wrap: step_hi = step_lo - 1 is 0 rows
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


# ---------------------------------------------------------------- v1 verifier
class _Rd:
    """bincode 1.3 fixint LE reader over a ProofV1 (proof.rs:80-98)."""

    def __init__(self, b: bytes):
        self.b, self.p = bytes(b), 0

    def take(self, n):
        if self.p + n > len(self.b):
            raise ValueError("truncated proof bytes")
        s = self.b[self.p:self.p + n]
        self.p += n
        return s

    def u64(self):
        return struct.unpack("<Q", self.take(8))[0]

    def vec32(self):
        return [self.take(32) for _ in range(self.u64())]


def _opening(rd):  # proof.rs:44-66
    return {"value_le": rd.take(8), "index": rd.u64(), "chunk_index": rd.u64(), "index_in_chunk": rd.u64(),
            "chunk_root": rd.take(32), "path_in_chunk": rd.vec32(), "path_to_chunk": rd.vec32()}


def parse_proof_v1(b: bytes) -> dict:
    rd = _Rd(b)
    pf = {"domain_n": rd.u64(), "tau": rd.u64(), "col_roots": []}
    for _ in range(rd.u64()):
        lab = rd.take(rd.u64()).decode()
        pf["col_roots"].append((lab, rd.take(32)))
    pf["queries"] = []
    for _ in range(rd.u64()):
        q = {"row": rd.u64(), "per_tape": []}
        for _ in range(rd.u64()):
            q["per_tape"].append({k: _opening(rd) for k in ("mv", "next_mv", "write_flag", "write_sym", "head",
                                                              "next_head", "win_len", "in_off", "out_off")})
        for k in ("is_first", "is_last", "input_mv"):
            q[k] = _opening(rd)
        pf["queries"].append(q)
    pf["fri_roots"] = rd.vec32()
    pf["fri_queries"] = []
    for _ in range(rd.u64()):
        pos = [rd.u64() for _ in range(rd.u64())]
        pairs = [(rd.take(8), rd.vec32(), rd.take(8), rd.vec32()) for _ in range(rd.u64())]
        pf["fri_queries"].append({"positions": pos, "pairs": pairs})
    pf["fri_final_value_le"] = rd.take(8)
    pf["manifest_root"] = rd.take(32)
    return pf


def merkle_verify(root, leaf_h, idx, sibs):  # merkle.rs:111-126 (MerkleTree::verify)
    cur = leaf_h
    for s in sibs:
        cur = h2(cur, s) if idx & 1 == 0 else h2(s, cur)
        idx >>= 1
    return cur == root


def _leaf_lab_raw(value_le: bytes, label: str):  # merkle.rs:132-147 over the opened bytes as given
    lb = label.encode()
    return blake3(b"col_leaf" + struct.pack("<I", len(lb)) + lb + bytes(value_le))


def verify_v1(proof_bytes: bytes, tau_blocks=None):
    """verify_v1 (crates/sezkp-stark/src/v1/verify.rs:60-196) with fri_verify
    (fri.rs:130-222) and verify_chunked_open (merkle.rs:243-280). Returns None
    when the proof is accepted, else the reference's error text. `tau_blocks`:
    the block windows' tau (verify.rs:73-81), or None for no blocks."""
    fe = lambda le: int.from_bytes(le, "little") % P
    try:
        pf = parse_proof_v1(proof_bytes)
    except ValueError as e:
        return str(e)
    if pf["domain_n"] % 8:
        return "FRI domain_n not multiple of blowup"
    n = pf["domain_n"] // 8
    if n == 0 or n & (n - 1):
        return "trace length n must be a power of two"
    tau = pf["tau"]
    if tau_blocks is not None and tau_blocks != tau:
        return f"tau mismatch vs. block windows: got {tau}, expected {tau_blocks}"
    tr = Transcript("sezkp-stark/v1")
    tr.absorb("manifest_root", pf["manifest_root"])
    tr.absorb_u64("n", n)
    tr.absorb_u64("tau", tau)
    tr.absorb_u64("n_cols", len(pf["col_roots"]))
    for _lab, r in pf["col_roots"]:
        tr.absorb("col_root", r)
    ab = tr.challenge("alphas", 64)
    a = [int.from_bytes(ab[8 * i:8 * i + 8], "little") % P for i in range(8)]
    tr.absorb("masks", b"masks")  # derive_mask_coeffs (masking.rs:56-79): alignment only
    tr.absorb_u64("n_masks", 1)
    tr.absorb_u64("deg", 4)
    for _ in range(4):
        tr.challenge("mask_coeff", 8)
    tr.challenge("ood_point", 8)
    roots = pf["fri_roots"]
    nl = len(roots)
    tr_rows = Transcript.__new__(Transcript)
    tr_rows.stream = tr.stream
    if nl > 0:
        tr_rows.absorb("fri_layer_root", roots[0])
        tr_rows.challenge("fri_betas", 8 * max(nl - 1, 0))
        for r in range(1, nl):
            tr_rows.absorb("fri_layer_root", roots[r])
    qb = tr_rows.challenge("row_queries", 8 * 30)
    expected = [int.from_bytes(qb[8 * i:8 * i + 8], "little") % max(n, 1) for i in range(30)]
    if len(expected) != len(pf["queries"]):
        return f"AIR query count mismatch (expected {len(expected)}, got {len(pf['queries'])})"
    for i, q in enumerate(pf["queries"]):
        if q["row"] != expected[i]:
            return f"AIR query row mismatch at position {i}: got {q['row']}, expected {expected[i]}"
    root_map = dict(pf["col_roots"])

    def vopen(label, o):
        if label not in root_map:
            return f"missing col root for {label}"
        lh = _leaf_lab_raw(o["value_le"], label)
        if not (merkle_verify(o["chunk_root"], lh, o["index_in_chunk"], o["path_in_chunk"])
                and merkle_verify(root_map[label], o["chunk_root"], o["chunk_index"], o["path_to_chunk"])):
            return f"chunked merkle path failed for column {label} @ {o['index']}"
        return None

    names = [("mv", "mv"), ("mv", "next_mv"), ("wflag", "write_flag"), ("wsym", "write_sym"), ("head", "head"),
             ("head", "next_head"), ("winlen", "win_len"), ("in_off", "in_off"), ("out_off", "out_off")]
    for q in pf["queries"]:
        for lab in ("input_mv", "is_first", "is_last"):
            e = vopen(lab, q[lab])
            if e:
                return e
        for r, t in enumerate(q["per_tape"]):
            for kind, key in names:
                e = vopen(f"{kind}_{r}", t[key])
                if e:
                    return e
        # compose_row_from_openings + compose_boundary_from_openings (air.rs:209-238)
        isf, isl = fe(q["is_first"]["value_le"]), fe(q["is_last"]["value_le"])
        acc = 0
        for t in q["per_tape"]:
            mv, flg, hd, hn, nmv = (fe(t[k]["value_le"]) for k in ("mv", "write_flag", "head", "next_head", "next_mv"))
            acc += a[0] * flg * (flg - 1) + a[1] * mv * (mv - 1) * (mv + 1) + a[2] * (1 - isl) * (hn - hd - nmv)
            acc += a[2] * isf * (hd - mv - fe(t["in_off"]["value_le"])) + a[2] * isl * (hd - fe(t["out_off"]["value_le"]))
        if acc % P:
            return f"AIR composition non-zero at row {q['row']}"
    # fri_verify (fri.rs:130-222), on the transcript after the OOD draw
    if nl == 0:
        return "no FRI roots"
    tr.absorb("fri_layer_root", roots[0])
    bb = tr.challenge("fri_betas", 8 * (nl - 1))
    betas = [int.from_bytes(bb[8 * i:8 * i + 8], "little") % P for i in range(nl - 1)]
    final = pf["fri_final_value_le"]
    if roots[nl - 1] != blake3(bytes(final)):
        return "final FRI value mismatch with last root"
    for fq in pf["fri_queries"]:
        pos, pairs = fq["positions"], fq["pairs"]
        if len(pos) != nl:
            return "positions length mismatch"
        if len(pairs) != nl - 1:
            return "pairs length mismatch"
        idx, ln = pos[0], 1 << (nl - 1)
        for l in range(nl - 1):
            half = ln // 2
            j = idx ^ half
            vi_le, pi, vj_le, pj = pairs[l]
            if not (merkle_verify(roots[l], blake3(vi_le), idx, pi) and merkle_verify(roots[l], blake3(vj_le), j, pj)):
                return f"FRI Merkle path failed at layer {l}"
            vi, vj = fe(vi_le), fe(vj_le)
            lower, upper = (vi, vj) if idx < half else (vj, vi)
            v_fold = (lower + betas[l] * upper) % P
            if pos[l + 1] != idx % half:
                return f"FRI index propagation failed at layer {l}"
            if l + 1 < nl - 1:
                if fe(pairs[l + 1][0]) != v_fold:
                    return f"FRI fold mismatch at layer {l}"
            elif struct.pack("<Q", v_fold) != bytes(final):
                return "final FRI value mismatch"
            idx, ln = idx % half, half
    return None
