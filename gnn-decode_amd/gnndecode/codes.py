"""Parity-check matrices of the codes the reference decodes (host-side, built natively).

* BCH(63,45)  — the reference loads it from classical/BCH(63,45).txt (classical/CGNNI.py:181).
  Here it is generated from its definition: narrow-sense binary BCH, n = 63, t = 3, over
  GF(2^6) with primitive polynomial x^6 + x + 1; g(x) = lcm(m1, m3, m5) (degree 18),
  h(x) = (x^63 + 1) / g(x) (degree 45); H row i = reversed h coefficients shifted by i.
  tests/test_codes.py checks it equals the reference file bit for bit (golden fixture).
* Toric code (distance L) — restatement of quantum/error_generate.py:39-132 `generate_PCM`
  (the returned H; H_one is unused by the hot path).  Rows: L^2-1 Z-type then L^2-1 X-type
  plaquette checks on 2 L^2 edge qubits, symplectic columns [X part | Z part].
* 802.11n LDPC(648,324), rate 1/2, Z = 27 — NOT in the reference:
  built from the base matrix recorded there, flagged unverified; checks in tests.

All matrices are returned as H[V, C] (variables x checks), the orientation the reference
passes to `H.to_sparse()` (classical/CGNNI.py:181 `.t()`, quantum/decoder_v2_4.py:189).
"""
import numpy as np


# ---------------------------------------------------------------------------------------
# BCH
# ---------------------------------------------------------------------------------------
def _gf2m_tables(m, prim):
    n = (1 << m) - 1
    exp = [0] * (2 * n)
    x = 1
    for i in range(n):
        exp[i] = x
        x <<= 1
        if x >> m:
            x ^= prim
    for i in range(n, 2 * n):
        exp[i] = exp[i - n]
    log = [0] * (n + 1)
    for i in range(n):
        log[exp[i]] = i
    return exp, log


def _minimal_poly(i, m, exp, log):
    n = (1 << m) - 1
    conj = sorted({(i << k) % n for k in range(m)})
    poly = [1]                                   # coefficients over GF(2^m), low first
    for c in conj:                               # multiply by (x - alpha^c)
        r = exp[c]
        nxt = [0] * (len(poly) + 1)
        for d, a in enumerate(poly):
            nxt[d + 1] ^= a
            if a:
                nxt[d] ^= exp[(log[a] + log[r]) % n]
        poly = nxt
    assert all(p in (0, 1) for p in poly)
    return poly


def _pmul2(a, b):
    r = [0] * (len(a) + len(b) - 1)
    for i, x in enumerate(a):
        if x:
            for j, y in enumerate(b):
                r[i + j] ^= y
    return r


def _pdiv2(a, b):
    a = list(a)
    q = [0] * (len(a) - len(b) + 1)
    for i in range(len(a) - len(b), -1, -1):
        if a[i + len(b) - 1]:
            q[i] = 1
            for j, y in enumerate(b):
                a[i + j] ^= y
    if any(a):
        raise ValueError('non-zero remainder')
    return q


def bch_parity_check(m=6, t=3, prim=0b1000011):
    """Cyclic parity-check matrix H[C, n] of the narrow-sense binary BCH(n, k) code."""
    n = (1 << m) - 1
    exp, log = _gf2m_tables(m, prim)
    g = [1]
    seen = set()
    for i in range(1, 2 * t, 2):
        mp = tuple(_minimal_poly(i, m, exp, log))
        if mp not in seen:
            seen.add(mp)
            g = _pmul2(g, list(mp))
    h = _pdiv2([1] + [0] * (n - 1) + [1], g)
    k = len(h) - 1
    rows = n - k
    H = np.zeros((rows, n), np.uint8)
    pat = np.array(h[::-1], np.uint8)
    for i in range(rows):
        H[i, i:i + k + 1] = pat
    return H


def bch_63_45():
    """H[V=63, C=18] as the reference uses it (classical/CGNNI.py:181)."""
    return bch_parity_check(6, 3, 0b1000011).T.copy()


# ---------------------------------------------------------------------------------------
# toric code
# ---------------------------------------------------------------------------------------
def toric_code(L):
    """H[V = 4 L^2, C = 2 L^2 - 2] of the distance-L toric code, restating
    quantum/error_generate.py:39-132.  Plaquette i (< L^2 - 1) sits at grid position
    j = 2 L (i // L) + (i % L) of the 2L x L edge lattice; its Z check touches qubits
    j, j+L, (j+2L) mod 2L^2 and its right neighbour, its X check (offset 2L^2 in the
    symplectic vector) touches j, j+L, (j-L) mod 2L^2 and its left neighbour."""
    n = 2 * L * L
    g = L * L - 1
    H = np.zeros((2 * g, 2 * n), np.uint8)
    for i in range(g):
        r, col = divmod(i, L)
        j = 2 * L * r + col
        right = j + L + 1 if col != L - 1 else j + 1
        left = j - 1 if col != 0 else j - 1 + L
        for q in (j, j + L, (j + 2 * L) % n, right):
            H[i, q] = 1
        for q in (j, j + L, (j - L) % n, left):
            H[g + i, n + q] = 1
    return H.T.copy()


def toric_edge_types(L):
    """Edge type in [0, 8) of every edge of toric_code(L), in reference edge order (sorted
    by (v, c): H.to_sparse()._indices()).  Restates the `H_prime` labels that
    quantum/error_generate.py:92-124 writes beside H (0.2, 1, 2, 3 for a Z check's qubits
    j, j+L, right, (j+2L) mod 2L^2; 4.2, 5, 6, 7 for an X check's (j-L) mod 2L^2, left, j,
    j+L; `.long()` truncates to 0..7) — the one-hot edge features of
    quantum/decoder_v2_2.py:226-250.  (The shipped generate_PCM returns a different
    matrix, `H_one`, with labels up to 31, as its second value.)"""
    n = 2 * L * L
    g = L * L - 1
    label = {}
    for i in range(g):
        r, col = divmod(i, L)
        j = 2 * L * r + col
        right = j + L + 1 if col != L - 1 else j + 1
        left = j - 1 if col != 0 else j - 1 + L
        for q, t in ((j, 0), (j + L, 1), (right, 2), ((j + 2 * L) % n, 3)):
            label[(q, i)] = t
        for q, t in (((j - L) % n, 4), (left, 5), (j, 6), (j + L, 7)):
            label[(n + q, g + i)] = t
    H = toric_code(L)
    vs, cs = np.nonzero(H)                 # row-major: sorted by (v, c)
    return np.array([label[(int(v), int(c))] for v, c in zip(vs, cs)], np.int64)


# ---------------------------------------------------------------------------------------
# 802.11n LDPC(648, 324), Z = 27 (UNVERIFIED base matrix)
# ---------------------------------------------------------------------------------------
_WIFI_648_R12 = """
 0  -  -  -  0  0  -  -  0  -  -  0  1  0  -  -  -  -  -  -  -  -  -  -
22  0  -  - 17  -  0  0 12  -  -  -  -  0  0  -  -  -  -  -  -  -  -  -
 6  -  0  - 10  -  -  - 24  -  0  -  -  -  0  0  -  -  -  -  -  -  -  -
 2  -  -  0 20  -  -  - 25  0  -  -  -  -  -  0  0  -  -  -  -  -  -  -
23  -  -  -  3  -  -  -  0  -  9 11  -  -  -  -  0  0  -  -  -  -  -  -
24  - 23  1 17  -  3  - 10  -  -  -  -  -  -  -  -  0  0  -  -  -  -  -
25  -  -  -  8  -  -  -  7 18  -  -  0  -  -  -  -  -  0  0  -  -  -  -
13 24  -  -  0  -  8  -  6  -  -  -  -  -  -  -  -  -  -  0  0  -  -  -
 7 20  - 16 22 10  -  - 23  -  -  -  -  -  -  -  -  -  -  -  0  0  -  -
11  -  -  - 19  -  -  - 13  -  3 17  -  -  -  -  -  -  -  -  -  0  0  -
25  -  8  - 23 18  - 14  9  -  -  -  -  -  -  -  -  -  -  -  -  -  0  0
 3  -  -  - 16  -  -  2 25  5  -  -  1  -  -  -  -  -  -  -  -  -  -  0
"""


def wifi_ldpc_648():
    """H[V=648, C=324] expanded from the 12x24 base matrix (cyclic shifts of I_27)."""
    Z = 27
    base = [row.split() for row in _WIFI_648_R12.strip().splitlines()]
    Hc = np.zeros((12 * Z, 24 * Z), np.uint8)
    I = np.eye(Z, dtype=np.uint8)
    for r, row in enumerate(base):
        for c, s in enumerate(row):
            if s != '-':
                Hc[r * Z:(r + 1) * Z, c * Z:(c + 1) * Z] = np.roll(I, int(s), axis=1)
    return Hc.T.copy()


def gf2_rank(M):
    A = np.array(M, np.uint8) % 2
    rank = 0
    rows, cols = A.shape
    for c in range(cols):
        piv = np.nonzero(A[rank:, c])[0]
        if piv.size == 0:
            continue
        p = rank + piv[0]
        A[[rank, p]] = A[[p, rank]]
        mask = A[:, c].astype(bool)
        mask[rank] = False
        A[mask] ^= A[rank]
        rank += 1
        if rank == rows:
            break
    return rank


def gf2_generator(H):
    """Generator matrix G [k, V] of the code {c : c H = 0 (mod 2)} for H [V, C] (the
    reference's orientation): a basis of the GF(2) null space of H^T by Gauss-Jordan
    elimination.  k = V - rank(H) (BCH(63,45): 45)."""
    A = np.array(H, np.uint8).T % 2                     # [C, V]
    rows, V = A.shape
    piv_cols, r = [], 0
    for c in range(V):
        piv = np.nonzero(A[r:, c])[0]
        if piv.size == 0:
            continue
        p = r + piv[0]
        A[[r, p]] = A[[p, r]]
        mask = A[:, c].astype(bool)
        mask[r] = False
        A[mask] ^= A[r]
        piv_cols.append(c)
        r += 1
        if r == rows:
            break
    free = [c for c in range(V) if c not in set(piv_cols)]
    G = np.zeros((len(free), V), np.uint8)
    for i, f in enumerate(free):                        # free variable f = 1, pivots solved
        G[i, f] = 1
        for j, pc in enumerate(piv_cols):
            G[i, pc] = A[j, f]
    return G


CODES = {
    'bch_63_45': bch_63_45,
    'toric_4': lambda: toric_code(4),
    'toric_5': lambda: toric_code(5),
    'toric_7': lambda: toric_code(7),
    'ldpc_648_324': wifi_ldpc_648,
}


def get_code(name):
    if name.startswith('toric_'):
        return toric_code(int(name.split('_')[1]))
    return CODES[name]()


# ---------------------------------------------------------------------------------------
# toric logical operators (for the training loss and FER metric)
# ---------------------------------------------------------------------------------------
def _symplectic(a, b):
    n = a.size // 2
    return int(np.dot(a, np.concatenate([b[n:], b[:n]])) % 2)


def toric_logicals(H):
    """Logical operators [4, V] of the code with parity-check matrix H[V, C], restating the
    reference's construction exactly (quantum/error_generate.py:145-248: `H_Prep`
    Gauss-Jordan with its column-exchange bookkeeping, then `get_logical`'s pairing of
    rows with symplectic product 1).  The loss (quantum/decoder_v2_4.py:314-315) sums
    |sin(pi/2 * L (e + e_hat))| per row, so the specific basis matters, not only its span."""
    Hc = (np.asarray(H) != 0).T.astype(np.int64)        # [C, V] as H_Prep(H.t()) receives it
    rows, cols = Hc.shape
    Hp = Hc.copy()
    exchange = []
    for i in range(rows):                                # H_Prep.Get_Identity
        if Hp[i, i] != 1:
            for j in range(i, cols):
                if Hp[i, j] == 1:
                    Hp[:, [i, j]] = Hp[:, [j, i]]
                    exchange.append((i, j))
        for j in range(rows):
            if Hp[j, i] == 1 and i != j:
                Hp[j, :] = (Hp[i, :] + Hp[j, :]) % 2
    exchange.reverse()
    P = np.concatenate([Hp[:, rows:cols], np.eye(cols - rows, dtype=np.int64)], axis=0)
    for a, b in exchange:                                # H_Prep.get_H_Prep
        P[[a, b], :] = P[[b, a], :]
    P = np.concatenate([P[cols // 2:cols, :], P[0:cols // 2, :]], axis=0).T.copy()
    prows = P.shape[0]
    logical = []                                         # indices into P (rows never change
                                                         # once chosen: they match themselves)

    def is_logical(k):
        return any((P[k] == P[l]).all() for l in logical)

    for i in range(prows):                               # H_Prep.get_logical
        if is_logical(i):
            continue
        for j in range(i + 1, prows):
            if is_logical(j) or _symplectic(P[i], P[j]) != 1:
                continue
            logical += [i, j]
            for k in range(j + 1, prows):
                if not is_logical(k) and _symplectic(P[i], P[k]) == 1:
                    P[k] = (P[k] + P[j]) % 2
            for m in range(i + 1, prows):
                if not is_logical(m) and _symplectic(P[j], P[m]) == 1:
                    P[m] = (P[m] + P[i]) % 2
            break
    return np.stack([P[l] for l in logical]).astype(np.uint8)
