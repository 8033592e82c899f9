"""The fingerprint view's input: dataset.py:37-45 concatenates, per molecule,

    MACCS keys (167)  AllChem.GetMACCSKeysFingerprint(mol)
    ErG (441)         AllChem.GetErGFingerprint(mol, fuzzIncrement=0.3, maxPath=21, minPath=1)
    PubChem (881)     pubchemfp.GetPubChemFPs(mol)
    Morgan r2 (1024)  AllChem.GetMorganFingerprintAsBitVect(mol, 2, nBits=1024)

= 2,513 floats.  RDKit (rdkit==2022.9.3, README.md:10-19) is absent from the image, so this
module restates the four families over the molecules of mvml_gat.featurize (the same parser /
sanitiser the graph view uses), with its own SMARTS parser and substructure matcher:

* MACCS: the 166 public MACCS key SMARTS as RDKit's MACCSkeys module defines them, count
  thresholds "more than n unique matches", keys 125 (aromatic rings > 1) and 166 (fragments > 1)
  computed directly, keys 1 (isotope) and 44 (other) left unset as RDKit's SMARTS table does;
* PubChem: the 733 substructure keys of the public PubChem specification (the reference's own
  table, pubchemfp.py:28-733, loaded from data/pubchem_smarts.json) matched on the molecule
  with explicit hydrogens (Chem.AddHs, pubchemfp.py:1518), and the ring-count keys 116-263
  restated from pubchemfp.py:815-1511 over the SSSR rings;
* Morgan / ECFP4: RDKit's connectivity invariants (atomic number, degree, total H, charge,
  delta mass, ring membership) hashed with boost::hash_combine, radius-2 iterations over
  bond-type-labelled sorted neighbourhoods, duplicate environments dropped, bit = hash % 1024;
* ErG: the extended reduced graph of Stiefl et al. (J. Chem. Inf. Model. 2006): rings collapsed
  to aromatic / non-aromatic nodes, donor / acceptor / positive / negative property points,
  21 property-pair types x 21 topological distances with the 0.3 fuzzy increment.

Agreement with RDKit is **parity unpinned** (RDKit cannot run here); each family is pinned by
known answers in tests/test_fingerprints.py — the MACCS doctest vectors RDKit ships (and the
reference copies into pubchemfp.py:788-793) and hand-derived cases for the others.
Host-side data preparation, as in the reference (per item on the CPU).
"""
import json
import os
from functools import lru_cache

import numpy as np

from . import featurize as fz

MACCS_BITS, ERG_BITS, PUBCHEM_BITS, MORGAN_BITS = 167, 441, 881, 1024
FP_SIZE = MACCS_BITS + ERG_BITS + PUBCHEM_BITS + MORGAN_BITS  # 2513 (model.py:146, config.py)

_SYMBOLS = ("* H He Li Be B C N O F Ne Na Mg Al Si P S Cl Ar K Ca Sc Ti V Cr Mn Fe Co Ni Cu Zn Ga "
            "Ge As Se Br Kr Rb Sr Y Zr Nb Mo Tc Ru Rh Pd Ag Cd In Sn Sb Te I Xe Cs Ba La Ce Pr Nd "
            "Pm Sm Eu Gd Tb Dy Ho Er Tm Yb Lu Hf Ta W Re Os Ir Pt Au Hg Tl Pb Bi Po At Rn Fr Ra Ac "
            "Th Pa U Np Pu Am Cm Bk Cf Es Fm Md No Lr Rf").split()
_Z = {s: z for z, s in enumerate(_SYMBOLS)}
_AROM_SYM = {"c": 6, "n": 7, "o": 8, "s": 16, "p": 15, "b": 5, "se": 34, "as": 33, "te": 52}
SINGLE, DOUBLE, TRIPLE, AROMATIC = 1, 2, 3, fz.AROM


# ----------------------------------------------------------------------------------------------
# molecule view for matching
# ----------------------------------------------------------------------------------------------
class FPMol:
    """Atoms / bonds with the properties SMARTS primitives read.  add_hs: hydrogens as explicit
    atoms (Chem.AddHs); a heavy atom's total H count then comes from its H neighbours."""

    def __init__(self, m, add_hs=False):
        n0 = m.num_atoms
        self.z = [_Z[s] if s in _Z else fz._ELEM[s][0] for s in m.sym]
        self.arom = list(m.arom)
        self.charge = list(m.charge)
        self.implicit = [m.total_h(i) for i in range(n0)]  # H not present as atoms
        self.bonds = [(a, b, o) for (a, b, o) in m.bonds]
        if add_hs:
            for i in range(n0):
                for _ in range(self.implicit[i]):
                    j = len(self.z)
                    self.z.append(1)
                    self.arom.append(False)
                    self.charge.append(0)
                    self.implicit.append(0)
                    self.bonds.append((i, j, SINGLE))
                self.implicit[i] = 0
        n = len(self.z)
        self.n = n
        self.adj = [[] for _ in range(n)]
        for k, (a, b, _) in enumerate(self.bonds):
            self.adj[a].append((b, k))
            self.adj[b].append((a, k))
        rings = fz._sssr(m)  # explicit H never sit in rings: the heavy-atom SSSR is the SSSR
        self.rings = rings
        self.ring_count = [0] * n
        self.ring_sizes = [set() for _ in range(n)]
        self.bond_ring = [False] * len(self.bonds)
        for atoms, bonds in rings:
            for a in atoms:
                self.ring_count[a] += 1
                self.ring_sizes[a].add(len(atoms))
            for k in bonds:
                self.bond_ring[k] = True
        self.ring_bonds_of = [sum(1 for (_, k) in self.adj[i] if self.bond_ring[k]) for i in range(n)]

    def total_h(self, i):
        return self.implicit[i] + sum(1 for (j, _) in self.adj[i] if self.z[j] == 1)

    def degree(self, i):
        return len(self.adj[i])

    def valence(self, i):
        v = self.implicit[i]
        for (_, k) in self.adj[i]:
            o = self.bonds[k][2]
            v += 1.5 if o == AROMATIC else o
        return int(round(v))

    def bond_between(self, a, b):
        for (j, k) in self.adj[a]:
            if j == b:
                return k
        return -1


# ----------------------------------------------------------------------------------------------
# SMARTS
# ----------------------------------------------------------------------------------------------
class Query:
    def __init__(self):
        self.atoms = []   # predicates (mol, i) -> bool
        self.keys = []    # the atom's SMARTS text: candidate lists are cached per molecule by it
        self.bonds = []   # (a, b, predicate (mol, k) -> bool)
        self.adj = []
        self.plan = None

    def add_atom(self, pred, key):
        self.atoms.append(pred)
        self.keys.append(key)
        self.adj.append([])
        return len(self.atoms) - 1

    def add_bond(self, a, b, pred):
        self.bonds.append((a, b, pred))
        k = len(self.bonds) - 1
        self.adj[a].append((b, k))
        self.adj[b].append((a, k))


def _num(s, i, default):
    j = i
    while j < len(s) and s[j].isdigit():
        j += 1
    return (int(s[i:j]) if j > i else default), j


def _bond_default(m, k):
    return m.bonds[k][2] in (SINGLE, AROMATIC)


_BOND_PRIM = {
    "-": lambda m, k: m.bonds[k][2] == SINGLE,
    "=": lambda m, k: m.bonds[k][2] == DOUBLE,
    "#": lambda m, k: m.bonds[k][2] == TRIPLE,
    ":": lambda m, k: m.bonds[k][2] == AROMATIC,
    "~": lambda m, k: True,
    "@": lambda m, k: m.bond_ring[k],
    "/": lambda m, k: m.bonds[k][2] == SINGLE,
    "\\": lambda m, k: m.bonds[k][2] == SINGLE,
}


def _logic(terms, ops):
    """Fold primitive predicates by SMARTS precedence: '!' (unary, bound at tokenising),
    '&' / implicit (high), ',' (or), ';' (low and)."""
    def fold(items, op):
        if len(items) == 1:
            return items[0]
        if op == "or":
            return lambda m, i, fs=tuple(items): any(f(m, i) for f in fs)
        return lambda m, i, fs=tuple(items): all(f(m, i) for f in fs)

    # split by ';' then ',' then '&'
    groups_low, cur_low = [], [[]]
    for t, op in zip(terms, ops + [None]):
        cur_low[-1].append(t)
        if op == ";":
            groups_low.append(cur_low)
            cur_low = [[]]
        elif op == ",":
            cur_low.append([])
    groups_low.append(cur_low)
    lows = []
    for ors in groups_low:
        lows.append(fold([fold(ands, "and") for ands in ors], "or"))
    return fold(lows, "and")


def _parse_atom_expr(s, recurse):
    """Bracket-atom expression -> predicate (mol, i)."""
    if s == "H" or (s.startswith("H") and len(s) > 1 and s[1] in "+-"):
        ch = 0
        if len(s) > 1:
            sign = 1 if s[1] == "+" else -1
            mag, _ = _num(s, 2, 1)
            ch = sign * mag
        return lambda m, i, c=ch: m.z[i] == 1 and m.charge[i] == c
    terms, ops = [], []
    i, neg, expect_term = 0, False, True
    while i < len(s):
        c = s[i]
        if c in ";,&":
            ops.append(c if c != "&" else "&")
            i += 1
            expect_term = True
            continue
        if c == "!":
            neg = not neg
            i += 1
            continue
        if not expect_term:  # implicit '&' between adjacent primitives
            ops.append("&")
        f, i = _atom_primitive(s, i, recurse)
        if neg:
            f = (lambda g: lambda m, a: not g(m, a))(f)
            neg = False
        terms.append(f)
        expect_term = False
    return _logic(terms, ops)


def _atom_primitive(s, i, recurse):
    c = s[i]
    t2 = s[i:i + 2]
    if c.isupper() and len(t2) == 2 and t2[1].islower() and t2 in _Z:  # Hf, Rb, Dy, Xe, Cl, ...
        return (lambda m, a, z=_Z[t2]: m.z[a] == z and not m.arom[a]), i + 2
    if c == "*":
        return (lambda m, a: True), i + 1
    if c == "$":
        depth, j = 0, i + 1
        while True:
            if s[j] == "(":
                depth += 1
            elif s[j] == ")":
                depth -= 1
                if depth == 0:
                    break
            j += 1
        sub = recurse(s[i + 2:j])
        return (lambda m, a, q=sub: _anchored(q, m, a)), j + 1
    if c == "#":
        n, j = _num(s, i + 1, 0)
        return (lambda m, a, n=n: m.z[a] == n), j
    if c in "+-":
        sign = 1 if c == "+" else -1
        j = i + 1
        if j < len(s) and s[j].isdigit():
            mag, j = _num(s, j, 1)
        else:
            mag = 1
            while j < len(s) and s[j] == c:
                mag += 1
                j += 1
        return (lambda m, a, v=sign * mag: m.charge[a] == v), j
    if c == "H":
        n, j = _num(s, i + 1, 1)
        return (lambda m, a, n=n: m.total_h(a) == n), j
    if c == "h":
        n, j = _num(s, i + 1, 1)
        return (lambda m, a, n=n: m.implicit[a] == n), j
    if c == "D":
        n, j = _num(s, i + 1, 1)
        return (lambda m, a, n=n: m.degree(a) == n), j
    if c == "X":
        n, j = _num(s, i + 1, 1)
        return (lambda m, a, n=n: m.degree(a) + m.implicit[a] == n), j
    if c == "v":
        n, j = _num(s, i + 1, 1)
        return (lambda m, a, n=n: m.valence(a) == n), j
    if c == "x":
        n, j = _num(s, i + 1, None)
        if n is None:
            return (lambda m, a: m.ring_bonds_of[a] > 0), j
        return (lambda m, a, n=n: m.ring_bonds_of[a] == n), j
    if c == "R":
        n, j = _num(s, i + 1, None)
        if n is None:
            return (lambda m, a: m.ring_count[a] > 0), j
        return (lambda m, a, n=n: m.ring_count[a] == n), j
    if c == "r":
        n, j = _num(s, i + 1, None)
        if n is None:
            return (lambda m, a: m.ring_count[a] > 0), j
        return (lambda m, a, n=n: n in m.ring_sizes[a]), j
    if c == "a" and not s[i:i + 2] in ("as", "al", "ag", "ar", "at", "am", "ac", "au"):
        return (lambda m, a: m.arom[a]), i + 1
    if c == "A" and not (i + 1 < len(s) and s[i + 1].islower()):
        return (lambda m, a: not m.arom[a]), i + 1
    # element symbols: aromatic lowercase, or aliphatic (two letters when valid)
    for L in (2, 1):
        t = s[i:i + L]
        if len(t) == L and t in _AROM_SYM:
            return (lambda m, a, z=_AROM_SYM[t]: m.z[a] == z and m.arom[a]), i + L
    for L in (2, 1):
        t = s[i:i + L]
        if len(t) == L and t[0].isupper() and t in _Z:
            return (lambda m, a, z=_Z[t]: m.z[a] == z and not m.arom[a]), i + L
    raise ValueError(f"unsupported SMARTS primitive at {s[i:]!r}")


def _parse_bond_expr(s):
    terms, ops, neg = [], [], False
    expect = True
    for c in s:
        if c in ";,&":
            ops.append(c)
            expect = True
            continue
        if c == "!":
            neg = not neg
            continue
        if not expect:
            ops.append("&")
        f = _BOND_PRIM[c]
        if neg:
            f = (lambda g: lambda m, k: not g(m, k))(f)
            neg = False
        terms.append(f)
        expect = False
    return _logic(terms, ops)


_ORG_OUT = ("Cl", "Br", "B", "C", "N", "O", "P", "S", "F", "I")


@lru_cache(maxsize=None)
def parse_smarts(s):
    q = Query()
    i, prev, pending, stack, rings = 0, None, None, [], {}

    def link(a):
        nonlocal pending
        if prev is not None:
            q.add_bond(prev, a, pending or _bond_default)
        pending = None

    while i < len(s):
        c = s[i]
        if c == "(":
            stack.append(prev)
            i += 1
        elif c == ")":
            prev = stack.pop()
            i += 1
        elif c == ".":
            prev, pending = None, None
            i += 1
        elif c in "-=#:~@!/\\;&,":
            j = i
            while j < len(s) and s[j] in "-=#:~@!/\\;&,":
                j += 1
            pending = _parse_bond_expr(s[i:j])
            i = j
        elif c.isdigit() or c == "%":
            if c == "%":
                num, i = int(s[i + 1:i + 3]), i + 3
            else:
                num, i = int(c), i + 1
            if num in rings:
                a, bp = rings.pop(num)
                q.add_bond(a, prev, pending or bp or _bond_default)
                pending = None
            else:
                rings[num] = (prev, pending)
                pending = None
        elif c == "[":
            depth, j = 0, i
            while True:
                if s[j] == "[":
                    depth += 1
                elif s[j] == "]":
                    depth -= 1
                    if depth == 0:
                        break
                j += 1
            a = q.add_atom(_parse_atom_expr(s[i + 1:j], parse_smarts), s[i:j + 1])
            link(a)
            prev, i = a, j + 1
        else:
            if c == "*":
                pred, L = (lambda m, a: True), 1
            elif c == "a":
                pred, L = (lambda m, a: m.arom[a]), 1
            elif c == "A":
                pred, L = (lambda m, a: not m.arom[a]), 1
            elif s[i:i + 2] in ("Cl", "Br"):
                pred, L = (lambda m, a, z=_Z[s[i:i + 2]]: m.z[a] == z and not m.arom[a]), 2
            elif c in _AROM_SYM:
                pred, L = (lambda m, a, z=_AROM_SYM[c]: m.z[a] == z and m.arom[a]), 1
            elif c in _ORG_OUT:
                pred, L = (lambda m, a, z=_Z[c]: m.z[a] == z and not m.arom[a]), 1
            else:
                raise ValueError(f"unsupported SMARTS at {s[i:]!r} in {s!r}")
            a = q.add_atom(pred, s[i:i + L])
            link(a)
            prev, i = a, i + L
    if rings or stack:
        raise ValueError(f"unbalanced SMARTS {s!r}")
    return q


# ----------------------------------------------------------------------------------------------
# substructure matching (backtracking over a DFS order of the query)
# ----------------------------------------------------------------------------------------------
def _plan(q):
    order, parent, seen = [], {}, set()
    for root in range(len(q.atoms)):
        if root in seen:
            continue
        stack = [(root, None)]
        while stack:
            a, pb = stack.pop()
            if a in seen:
                continue
            seen.add(a)
            order.append(a)
            parent[a] = pb
            for (b, k) in reversed(q.adj[a]):
                if b not in seen:
                    stack.append((b, (a, k)))
    return order, parent


def _matches(q, m, first=None, limit=None):
    """Unique matches (atom sets) of q in m; first: the molecule atom query atom 0 must map to."""
    nq = len(q.atoms)
    cache = m.__dict__.setdefault("_cand", {})
    if q.plan is None:
        q.plan = _plan(q)
    order, parent = q.plan
    cands, cset_sets = [], []
    for a in range(nq):
        key = q.keys[a]
        if key not in cache:
            c = [i for i in range(m.n) if q.atoms[a](m, i)]
            cache[key] = (c, set(c))
        cands.append(cache[key][0])
        cset_sets.append(cache[key][1])
        if not cands[-1]:
            return set()
    mapping = [-1] * nq
    used = set()
    found = set()
    pos = {a: t for t, a in enumerate(order)}

    def ok_bonds(a, i):
        for (b, k) in q.adj[a]:
            if pos[b] < pos[a]:
                mb = m.bond_between(i, mapping[b])
                if mb < 0 or not q.bonds[k][2](m, mb):
                    return False
        return True

    def rec(t):
        if limit is not None and len(found) >= limit:
            return
        if t == nq:
            found.add(frozenset(mapping))
            return
        a = order[t]
        pb = parent[a]
        if pb is None:
            pool = cands[a] if not (first is not None and a == 0) else [first]
            cset = None
        else:
            pool = [j for (j, _) in m.adj[mapping[pb[0]]]]
            cset = cands[a]
        for i in pool:
            if i in used or (cset is not None and i not in cset_sets[a]):
                continue
            if pb is None and not q.atoms[a](m, i):
                continue
            if not ok_bonds(a, i):
                continue
            mapping[a] = i
            used.add(i)
            rec(t + 1)
            used.discard(i)
            mapping[a] = -1
            if limit is not None and len(found) >= limit:
                return

    rec(0)
    return found


def _anchored(q, m, i):
    cache = m.__dict__.setdefault("_rec", {})
    key = (id(q), i)
    if key not in cache:
        cache[key] = bool(_matches(q, m, first=i, limit=1))
    return cache[key]


def count_matches(smarts, m):
    return len(_matches(parse_smarts(smarts), m))


def has_match(smarts, m):
    return bool(_matches(parse_smarts(smarts), m, limit=1))


# ----------------------------------------------------------------------------------------------
# MACCS (RDKit MACCSkeys definitions)
# ----------------------------------------------------------------------------------------------
_R8 = ",".join("$([R]@1" + "@[R]" * (n - 1) + "1)" for n in range(8, 15))
MACCS_SMARTS = {
    2: ("[#104]", 0), 3: ("[#32,#33,#34,#50,#51,#52,#82,#83,#84]", 0),
    4: ("[Ac,Th,Pa,U,Np,Pu,Am,Cm,Bk,Cf,Es,Fm,Md,No,Lr]", 0), 5: ("[Sc,Ti,Y,Zr,Hf]", 0),
    6: ("[La,Ce,Pr,Nd,Pm,Sm,Eu,Gd,Tb,Dy,Ho,Er,Tm,Yb,Lu]", 0), 7: ("[V,Cr,Mn,Nb,Mo,Tc,Ta,W,Re]", 0),
    8: ("[!#6;!#1]1~*~*~*~1", 0), 9: ("[Fe,Co,Ni,Ru,Rh,Pd,Os,Ir,Pt]", 0),
    10: ("[Be,Mg,Ca,Sr,Ba,Ra]", 0), 11: ("*1~*~*~*~1", 0), 12: ("[Cu,Zn,Ag,Cd,Au,Hg]", 0),
    13: ("[#8]~[#7](~[#6])~[#6]", 0), 14: ("[#16]-[#16]", 0), 15: ("[#8]~[#6](~[#8])~[#8]", 0),
    16: ("[!#6;!#1]1~*~*~1", 0), 17: ("[#6]#[#6]", 0), 18: ("[#5,#13,#31,#49,#81]", 0),
    19: ("*1~*~*~*~*~*~*~1", 0), 20: ("[#14]", 0), 21: ("[#6]=[#6](~[!#6;!#1])~[!#6;!#1]", 0),
    22: ("*1~*~*~1", 0), 23: ("[#7]~[#6](~[#8])~[#8]", 0), 24: ("[#7]-[#8]", 0),
    25: ("[#7]~[#6](~[#7])~[#7]", 0), 26: ("[#6]=;@[#6](@*)@*", 0), 27: ("[I]", 0),
    28: ("[!#6;!#1]~[CH2]~[!#6;!#1]", 0), 29: ("[#15]", 0),
    30: ("[#6]~[!#6;!#1](~[#6])(~[#6])~*", 0), 31: ("[!#6;!#1]~[F,Cl,Br,I]", 0),
    32: ("[#6]~[#16]~[#7]", 0), 33: ("[#7]~[#16]", 0), 34: ("[CH2]=*", 0),
    35: ("[Li,Na,K,Rb,Cs,Fr]", 0), 36: ("[#16R]", 0), 37: ("[#7]~[#6](~[#8])~[#7]", 0),
    38: ("[#7]~[#6](~[#6])~[#7]", 0), 39: ("[#8]~[#16](~[#8])~[#8]", 0), 40: ("[#16]-[#8]", 0),
    41: ("[#6]#[#7]", 0), 42: ("F", 0), 43: ("[!#6;!#1;!H0]~*~[!#6;!#1;!H0]", 0),
    45: ("[#6]=[#6]~[#7]", 0), 46: ("Br", 0), 47: ("[#16]~*~[#7]", 0),
    48: ("[#8]~[!#6;!#1](~[#8])(~[#8])", 0), 49: ("[!+0]", 0), 50: ("[#6]=[#6](~[#6])~[#6]", 0),
    51: ("[#6]~[#16]~[#8]", 0), 52: ("[#7]~[#7]", 0), 53: ("[!#6;!#1;!H0]~*~*~*~[!#6;!#1;!H0]", 0),
    54: ("[!#6;!#1;!H0]~*~*~[!#6;!#1;!H0]", 0), 55: ("[#8]~[#16]~[#8]", 0),
    56: ("[#8]~[#7](~[#8])~[#6]", 0), 57: ("[#8R]", 0), 58: ("[!#6;!#1]~[#16]~[!#6;!#1]", 0),
    59: ("[#16]!:*:*", 0), 60: ("[#16]=[#8]", 0), 61: ("*~[#16](~*)~*", 0), 62: ("*@*!@*@*", 0),
    63: ("[#7]=[#8]", 0), 64: ("*@*!@[#16]", 0), 65: ("c:n", 0), 66: ("[#6]~[#6](~[#6])(~[#6])~*", 0),
    67: ("[!#6;!#1]~[#16]", 0), 68: ("[!#6;!#1;!H0]~[!#6;!#1;!H0]", 0),
    69: ("[!#6;!#1]~[!#6;!#1;!H0]", 0), 70: ("[!#6;!#1]~[#7]~[!#6;!#1]", 0), 71: ("[#7]~[#8]", 0),
    72: ("[#8]~*~*~[#8]", 0), 73: ("[#16]=*", 0), 74: ("[CH3]~*~[CH3]", 0), 75: ("*!@[#7]@*", 0),
    76: ("[#6]=[#6](~*)~*", 0), 77: ("[#7]~*~[#7]", 0), 78: ("[#6]=[#7]", 0),
    79: ("[#7]~*~*~[#7]", 0), 80: ("[#7]~*~*~*~[#7]", 0), 81: ("[#16]~*(~*)~*", 0),
    82: ("*~[CH2]~[!#6;!#1;!H0]", 0), 83: ("[!#6;!#1]1~*~*~*~*~1", 0), 84: ("[NH2]", 0),
    85: ("[#6]~[#7](~[#6])~[#6]", 0), 86: ("[C;H2,H3][!#6;!#1][C;H2,H3]", 0),
    87: ("[F,Cl,Br,I]!@*@*", 0), 88: ("[#16]", 0), 89: ("[#8]~*~*~*~[#8]", 0),
    90: ("[$([!#6;!#1;!H0]~*~*~[CH2]~*),$([!#6;!#1;!H0;R]1@[R]@[R]@[CH2;R]1),"
         "$([!#6;!#1;!H0]~[R]1@[R]@[CH2;R]1)]", 0),
    91: ("[$([!#6;!#1;!H0]~*~*~*~[CH2]~*),$([!#6;!#1;!H0;R]1@[R]@[R]@[R]@[CH2;R]1),"
         "$([!#6;!#1;!H0]~[R]1@[R]@[R]@[CH2;R]1),$([!#6;!#1;!H0]~*~[R]1@[R]@[CH2;R]1)]", 0),
    92: ("[#8]~[#6](~[#7])~[#6]", 0), 93: ("[!#6;!#1]~[CH3]", 0), 94: ("[!#6;!#1]~[#7]", 0),
    95: ("[#7]~*~*~[#8]", 0), 96: ("*1~*~*~*~*~1", 0), 97: ("[#7]~*~*~*~[#8]", 0),
    98: ("[!#6;!#1]1~*~*~*~*~*~1", 0), 99: ("[#6]=[#6]", 0), 100: ("*~[CH2]~[#7]", 0),
    101: ("[" + _R8 + "]", 0), 102: ("[!#6;!#1]~[#8]", 0), 103: ("Cl", 0),
    104: ("[!#6;!#1;!H0]~*~[CH2]~*", 0), 105: ("*@*(@*)@*", 0),
    106: ("[!#6;!#1]~*(~[!#6;!#1])~[!#6;!#1]", 0), 107: ("[F,Cl,Br,I]~*(~*)~*", 0),
    108: ("[CH3]~*~*~*~[CH2]~*", 0), 109: ("*~[CH2]~[#8]", 0), 110: ("[#7]~[#6]~[#8]", 0),
    111: ("[#7]~*~[CH2]~*", 0), 112: ("*~*(~*)(~*)~*", 0), 113: ("[#8]!:*:*", 0),
    114: ("[CH3]~[CH2]~*", 0), 115: ("[CH3]~*~[CH2]~*", 0),
    116: ("[$([CH3]~*~*~[CH2]~*),$([CH3]~*1~*~[CH2]1)]", 0), 117: ("[#7]~*~[#8]", 0),
    118: ("[$(*~[CH2]~[CH2]~*),$(*1~[CH2]~[CH2]1)]", 1), 119: ("[#7]=*", 0),
    120: ("[!#6;R]", 1), 121: ("[#7;R]", 0), 122: ("*~[#7](~*)~*", 0), 123: ("[#8]~[#6]~[#8]", 0),
    124: ("[!#6;!#1]~[!#6;!#1]", 0), 126: ("*!@[#8]!@*", 0), 127: ("*@*!@[#8]", 1),
    128: ("[$(*~[CH2]~*~*~*~[CH2]~*),$([R]1@[CH2;R]@[R]@[R]@[R]@[CH2;R]1),"
          "$(*~[CH2]~[R]1@[R]@[R]@[CH2;R]1),$(*~[CH2]~*~[R]1@[R]@[CH2;R]1)]", 0),
    129: ("[$(*~[CH2]~*~*~[CH2]~*),$([R]1@[CH2]@[R]@[R]@[CH2;R]1),$(*~[CH2]~[R]1@[R]@[CH2;R]1)]", 0),
    130: ("[!#6;!#1]~[!#6;!#1]", 1), 131: ("[!#6;!#1;!H0]", 1), 132: ("[#8]~*~[CH2]~*", 0),
    133: ("*@*!@[#7]", 0), 134: ("[F,Cl,Br,I]", 0), 135: ("[#7]!:*:*", 0), 136: ("[#8]=*", 1),
    137: ("[!C;!c;R]", 0), 138: ("[!#6;!#1]~[CH2]~*", 1), 139: ("[O;!H0]", 0), 140: ("[#8]", 3),
    141: ("[CH3]", 2), 142: ("[#7]", 1), 143: ("*@*!@[#8]", 0), 144: ("*!:*:*!:*", 0),
    145: ("*1~*~*~*~*~*~1", 1), 146: ("[#8]", 2), 147: ("[$(*~[CH2]~[CH2]~*),$([R]1@[CH2;R]@[CH2;R]1)]", 0),
    148: ("*~[!#6;!#1](~*)~*", 0), 149: ("[C;H3,H4]", 1), 150: ("*!@*@*!@*", 0), 151: ("[#7;!H0]", 0),
    152: ("[#8]~[#6](~[#6])~[#6]", 0), 153: ("[!#6;!#1]~[CH2]~*", 0), 154: ("[#6]=[#8]", 0),
    155: ("*!@[CH2]!@*", 0), 156: ("[#7]~*(~*)~*", 0), 157: ("[#6]-[#8]", 0), 158: ("[#6]-[#7]", 0),
    159: ("[#8]", 1), 160: ("[C;H3,H4]", 0), 161: ("[#7]", 0), 162: ("a", 0),
    163: ("*1~*~*~*~*~*~1", 0), 164: ("[#8]", 0), 165: ("[R]", 0),
}


def _key(smarts, count, m):
    q = parse_smarts(smarts)
    if count == 0:
        return bool(_matches(q, m, limit=1))
    return len(_matches(q, m, limit=count + 1)) > count


def _n_components(m):
    seen, comps = set(), 0
    for s in range(m.n):
        if s in seen:
            continue
        comps += 1
        stack = [s]
        seen.add(s)
        while stack:
            x = stack.pop()
            for (y, _) in m.adj[x]:
                if y not in seen:
                    seen.add(y)
                    stack.append(y)
    return comps


def maccs_keys(mol):
    """GetMACCSKeysFingerprint: 167 bits (bit 0 unused)."""
    m = FPMol(mol)
    bits = np.zeros(MACCS_BITS, dtype=np.float32)
    for k, (sm, cnt) in MACCS_SMARTS.items():
        bits[k] = _key(sm, cnt, m)
    arom_rings = sum(1 for (_, bonds) in m.rings if all(m.bonds[k][2] == AROMATIC for k in bonds))
    bits[125] = arom_rings > 1
    bits[166] = _n_components(m) > 1
    return bits


# ----------------------------------------------------------------------------------------------
# PubChem (881 bits)
# ----------------------------------------------------------------------------------------------
@lru_cache(maxsize=1)
def _pubchem_table():
    path = os.path.join(os.path.dirname(os.path.abspath(__file__)), "data", "pubchem_smarts.json")
    with open(path) as f:
        return [tuple(r) for r in json.load(f)["keys"]]


# ring classes of pubchemfp.py func_1..func_7 (bit column k - 1 of the 7-wide ring-count grid)
def _ring_classes(m, atoms, bonds):
    orders = [m.bonds[k][2] for k in bonds]
    zs = {m.z[a] for k in bonds for a in m.bonds[k][:2]}
    saturated = all(o == SINGLE for o in orders)
    aromatic = all(o == AROMATIC for o in orders)
    any_arom = any(o == AROMATIC for o in orders)
    carbon = zs == {6}
    nitrogen = 7 in zs
    hetero = any(z not in (1, 6) for z in zs)
    unsat_nonarom = (not saturated) and not any_arom
    return [True,                                           # 1: any ring
            saturated or (aromatic and carbon),             # 2
            saturated or (aromatic and nitrogen),           # 3
            saturated or (aromatic and hetero),             # 4
            unsat_nonarom and carbon,                       # 5
            unsat_nonarom and nitrogen,                     # 6
            unsat_nonarom and hetero]                       # 7


# ring size -> (first slot of the 7-wide grid, number of count thresholds)
_RING_SLOTS = {3: (0, 2), 4: (2, 2), 5: (4, 5), 6: (9, 5), 7: (14, 2), 8: (16, 2), 9: (18, 1), 10: (19, 1)}


def pubchem_ring_bits(m):
    """pubchemfp.py:815-1511 (bits 116-263 of the 881): 148 bits."""
    bits = np.zeros(148, dtype=np.float32)
    counts = [dict.fromkeys(range(3, 11), 0) for _ in range(7)]
    for atoms, bonds in m.rings:
        size = len(atoms)
        if size not in _RING_SLOTS:
            continue
        for c, yes in enumerate(_ring_classes(m, atoms, bonds)):
            if yes:
                counts[c][size] += 1
    for c in range(7):
        for size, (slot, nthr) in _RING_SLOTS.items():
            for t in range(min(counts[c][size], nthr)):
                bits[c + 7 * (slot + t)] = 1
    n_arom = sum(1 for (_, bonds) in m.rings if all(m.bonds[k][2] == AROMATIC for k in bonds))
    n_het = sum(1 for (_, bonds) in m.rings
                if any(m.z[a] not in (1, 6) for k in bonds for a in m.bonds[k][:2]))
    for t in range(min(n_arom, 4)):
        bits[140 + 2 * t] = 1
    for t in range(1, 5):  # the reference's equality tests (pubchemfp.py:1484-1493)
        if (n_arom >= 4 and n_het >= 4) if t == 4 else (n_arom == t and n_het == t):
            for u in range(t):
                bits[141 + 2 * u] = 1
    return bits


def pubchem_fp(mol):
    """GetPubChemFPs (pubchemfp.py:1514-1536): 881 bits on the molecule with explicit H."""
    m = FPMol(mol, add_hs=True)
    out = np.zeros(PUBCHEM_BITS, dtype=np.float32)
    table = _pubchem_table()
    for idx, (sm, cnt) in enumerate(table):
        bit = idx if idx < 115 else idx + 148
        try:
            out[bit] = _key(sm, cnt, m)
        except ValueError:
            out[bit] = 0  # a pattern the SMARTS parser cannot read never matches (RDKit: None)
    out[115:263] = pubchem_ring_bits(m)
    return out


# ----------------------------------------------------------------------------------------------
# Morgan / ECFP (RDKit MorganFingerprints, radius 2, 1024 bits)
# ----------------------------------------------------------------------------------------------
_MASK = (1 << 64) - 1


def _hash_combine(seed, v):
    """boost::hash_combine on a 64-bit std::size_t seed (integer hash = the value)."""
    v &= _MASK
    return (seed ^ ((v + 0x9E3779B9 + ((seed << 6) & _MASK) + (seed >> 2)) & _MASK)) & _MASK


def _hash_range(vals):
    seed = 0
    for v in vals:
        seed = _hash_combine(seed, v)
    return seed & 0xFFFFFFFF


_BOND_TYPE_ID = {SINGLE: 1, DOUBLE: 2, TRIPLE: 3, AROMATIC: 12}


def morgan_fp(mol, radius=2, nbits=MORGAN_BITS):
    m = FPMol(mol)
    n = m.n
    inv = []
    for i in range(n):
        comp = [m.z[i], m.degree(i) + m.implicit[i], m.total_h(i), m.charge[i], 0]
        if m.ring_count[i]:
            comp.append(1)
        inv.append(_hash_range(comp))
    bits = np.zeros(nbits, dtype=np.float32)
    for i in range(n):
        bits[inv[i] % nbits] = 1
    # environments: the bond set each atom's current invariant covers
    env = [frozenset() for _ in range(n)]
    seen = set()
    for layer in range(radius):
        new_inv, new_env, cands = [], [], []
        for i in range(n):
            nb = sorted((_BOND_TYPE_ID[m.bonds[k][2]], inv[j]) for (j, k) in m.adj[i])
            seed = _hash_combine(layer, inv[i])
            for bt, iv in nb:
                seed = _hash_combine(seed, bt)
                seed = _hash_combine(seed, iv)
            e = set(env[i])
            for (j, k) in m.adj[i]:
                e.add(k)
                e |= env[j]
            new_inv.append(seed & 0xFFFFFFFF)
            new_env.append(frozenset(e))
            cands.append((frozenset(e), seed & 0xFFFFFFFF, i))
        # an environment already seen (this or an earlier layer) adds no bit; ties of the same
        # bond set in one layer keep the smallest invariant (RDKit's neighbourhood dedup)
        cands.sort(key=lambda t: (len(t[0]), t[1], t[2]))
        for e, h, i in cands:
            if not e or e in seen:
                continue
            seen.add(e)
            bits[h % nbits] = 1
        inv, env = new_inv, new_env
    return bits


# ----------------------------------------------------------------------------------------------
# ErG (extended reduced graph; RDKit GetErGFingerprint defaults + the reference's arguments)
# ----------------------------------------------------------------------------------------------
ERG_TYPES = 6  # donor, acceptor, positive, negative, hydrophobic ring, aromatic ring
_ERG_FEATS = {
    0: ("[N,O;!H0;!$(*-[#6,#16,#15]=[O,S])]", "[n;!H0]"),                       # donor
    1: ("[O;H0;!$(O-[#6,#16,#15]=O)]", "[O;H1;!$(O-[#6,#16,#15]=O)]",            # acceptor
        "[n;H0;+0]", "[N;H0;X1,X2;+0]", "[N;+0;$(N-C=O)]"),
    2: ("[+;!$(*~[-])]", "[NX3;H2,H1,H0;+0;!$(N-[#6,#16]=[O,N,S]);!$(N-a);!$(N#*);!$(N=*)]",  # positive
        "[$([NH]=C(N)N)]"),
    3: ("[-;!$(*~[+])]", "[$([OH]-[#6,#16,#15]=O)]"),                             # negative
}


def _pair_index(a, b):
    if a > b:
        a, b = b, a
    return a * ERG_TYPES - a * (a - 1) // 2 + (b - a)


def erg_fp(mol, fuzz=0.3, min_path=1, max_path=21):
    m = FPMol(mol)
    feats = [set() for _ in range(m.n)]
    for t, pats in _ERG_FEATS.items():
        for sm in pats:
            q = parse_smarts(sm)
            for i in range(m.n):
                if q.atoms[0](m, i) and (len(q.atoms) == 1 or _anchored(q, m, i)):
                    feats[i].add(t)
    # reduced graph: every SSSR ring becomes one node (aromatic: type 5, else type 4) holding the
    # features of its atoms; atoms outside rings keep their own (possibly empty) feature sets
    node_of = [[] for _ in range(m.n)]
    nodes = []
    for atoms, bonds in m.rings:
        arom = all(m.bonds[k][2] == AROMATIC for k in bonds)
        f = {5 if arom else 4}
        for a in atoms:
            f |= feats[a]
            node_of[a].append(len(nodes))
        nodes.append(f)
    for i in range(m.n):
        if not node_of[i]:
            node_of[i].append(len(nodes))
            nodes.append(set(feats[i]))
    nn = len(nodes)
    adj = [set() for _ in range(nn)]
    for (a, b, _) in m.bonds:
        for u in node_of[a]:
            for v in node_of[b]:
                if u != v:
                    adj[u].add(v)
                    adj[v].add(u)
    for i in range(m.n):  # fused rings share atoms
        for u in node_of[i]:
            for v in node_of[i]:
                if u != v:
                    adj[u].add(v)
    out = np.zeros(ERG_BITS, dtype=np.float32)
    nbins = max_path - min_path + 1
    for u in range(nn):
        if not nodes[u]:
            continue
        dist = {u: 0}
        frontier = [u]
        while frontier:
            nxt = []
            for x in frontier:
                for y in adj[x]:
                    if y not in dist:
                        dist[y] = dist[x] + 1
                        nxt.append(y)
            frontier = nxt
        for v, d in dist.items():
            if v <= u or not nodes[v] or not (min_path <= d <= max_path):
                continue
            for a in nodes[u]:
                for b in nodes[v]:
                    base = _pair_index(a, b) * nbins
                    k = d - min_path
                    out[base + k] += 1.0
                    if k > 0:
                        out[base + k - 1] += fuzz
                    if k + 1 < nbins:
                        out[base + k + 1] += fuzz
    return out


# ----------------------------------------------------------------------------------------------
def fingerprint(smiles_or_mol):
    """dataset.py:37-45: [MACCS 167 | ErG 441 | PubChem 881 | Morgan r2 1024] as float32[2513]."""
    mol = fz.mol_from_smiles(smiles_or_mol) if isinstance(smiles_or_mol, str) else smiles_or_mol
    return np.concatenate([maccs_keys(mol), erg_fp(mol), pubchem_fp(mol), morgan_fp(mol)])


def fingerprints(smiles_list):
    """float32[len, 2513] (the fps_t tensor collate builds, dataset.py:56)."""
    return np.stack([fingerprint(s) for s in smiles_list]) if smiles_list else \
        np.zeros((0, FP_SIZE), dtype=np.float32)


def kegg_pool():
    """float32[420, 2513]: the fingerprints of the 420 KEGG test-split molecules
    (tests/golden/kegg_test_split.csv) as computed by fingerprints() and stored bit-packed in
    data/kegg_fp_pool.npz (tools/make_fp_pool.py) — real bit vectors for workloads whose
    molecules are synthetic (bench.py --workload mvp cycles them)."""
    import os
    path = os.path.join(os.path.dirname(os.path.abspath(__file__)), "data", "kegg_fp_pool.npz")
    with np.load(path, allow_pickle=False) as z:
        bits = np.unpackbits(z["bits"], axis=1, count=int(z["nbits"])).astype(np.float32)
        erg = z["erg"].astype(np.float32)
    return np.concatenate([bits[:, :MACCS_BITS], erg, bits[:, MACCS_BITS:]], axis=1)
