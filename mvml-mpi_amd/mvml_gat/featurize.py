"""SMILES -> molecule graph with dgllife's CanonicalAtomFeaturizer.

Replaces, for the graph view only, the reference's per-item featurisation
``Chem.MolFromSmiles(smiles)`` + ``mol_to_bigraph(mol, add_self_loop=True,
node_featurizer=CanonicalAtomFeaturizer('h'))`` (dataset.py:23, 33-35).  RDKit 2022.9.3 and
dgllife 0.3.0 (README.md:10-19) are absent from the image, so this module restates the parts
of RDKit's sanitisation that the 74 atom features depend on:

* SMILES parsing (organic subset, bracket atoms with H count / charge, branches, ring
  closures, explicit bond symbols, aromatic lowercase atoms);
* implicit hydrogens (default valences, RDKit's aromatic accumulation rule);
* kekulisation of aromatic input (perfect matching on the atoms that need a double bond);
* radicals of bracket atoms (RDKit assignRadicals);
* aromaticity perception, RDKit default model: SSSR rings (Horton minimum cycle basis) and
  fused pairs/triples of rings, per-atom pi-electron donor types, Hückel 4n+2;
* conjugation (RDKit markConjAtomBonds) and hybridisation from bonds + lone pairs;
* the 74-d feature vector in dgllife's order: atom type one-hot (43) | degree 0-10 (11) |
  implicit valence 0-6 (7) | formal charge | radical electrons | hybridisation SP..SP3D2 (5) |
  aromatic | total H 0-4 (5).

Host-side data preparation (the reference runs it per item on the CPU as well); everything it
produces is plain integer/float arrays that ``batching.bigraph_from_bonds`` turns into a graph.

* canonical atom order (dgllife's ``canonical_atom_order=True``): RDKit's canonical ranking
  restated (``canonical_ranks``) and applied as dgllife applies it.

Known differences from the reference:
* agreement with RDKit itself is **unpinned** (including the canonical ranks: tie-breaking
  details of RDKit's implementation cannot be checked; the view is permutation-invariant per
  molecule — GAT equivariant, Set2Set / GraphNorm invariant, KAT 4 in tests/test_oracle_kat.py —
  so a different canonical order only changes floating-point summation order);
* the rest of the agreement with RDKit is **unpinned** (RDKit cannot be run here); the restatement is
  pinned by hand-derived known answers in tests/test_featurize.py.
"""
import numpy as np

# dgllife CanonicalAtomFeaturizer atom_type_one_hot allowable set (43, encode_unknown=False)
ATOM_TYPES = ['C', 'N', 'O', 'S', 'F', 'Si', 'P', 'Cl', 'Br', 'Mg', 'Na', 'Ca', 'Fe', 'As', 'Al',
              'I', 'B', 'V', 'K', 'Tl', 'Yb', 'Sb', 'Sn', 'Ag', 'Pd', 'Co', 'Se', 'Ti', 'Zn', 'H',
              'Li', 'Ge', 'Cu', 'Au', 'Ni', 'Cd', 'In', 'Mn', 'Zr', 'Cr', 'Pt', 'Hg', 'Pb']
FEAT_SIZE = 74
HYB_SP, HYB_SP2, HYB_SP3, HYB_SP3D, HYB_SP3D2, HYB_S, HYB_UNSPEC = range(7)

# symbol -> (Z, outer electrons, allowed valences (RDKit atomic_data; -1 = any), Pauling EN)
_ELEM = {
    '*': (0, 0, (-1,), 0.0), 'H': (1, 1, (1,), 2.20), 'Li': (3, 1, (1, -1), 0.98),
    'B': (5, 3, (3,), 2.04), 'C': (6, 4, (4,), 2.55), 'N': (7, 5, (3,), 3.04),
    'O': (8, 6, (2,), 3.44), 'F': (9, 7, (1,), 3.98), 'Na': (11, 1, (1, -1), 0.93),
    'Mg': (12, 2, (2, -1), 1.31), 'Al': (13, 3, (3, -1), 1.61), 'Si': (14, 4, (4,), 1.90),
    'P': (15, 5, (3, 5, 7), 2.19), 'S': (16, 6, (2, 4, 6), 2.58), 'Cl': (17, 7, (1,), 3.16),
    'K': (19, 1, (1, -1), 0.82), 'Ca': (20, 2, (2, -1), 1.00), 'Ti': (22, 4, (-1,), 1.54),
    'V': (23, 5, (-1,), 1.63), 'Cr': (24, 6, (-1,), 1.66), 'Mn': (25, 7, (-1,), 1.55),
    'Fe': (26, 8, (-1,), 1.83), 'Co': (27, 9, (-1,), 1.88), 'Ni': (28, 10, (-1,), 1.91),
    'Cu': (29, 11, (-1,), 1.90), 'Zn': (30, 2, (-1,), 1.65), 'Ge': (32, 4, (4,), 2.01),
    'As': (33, 5, (3, 5, 7), 2.18), 'Se': (34, 6, (2, 4, 6), 2.55), 'Br': (35, 7, (1,), 2.96),
    'Zr': (40, 4, (-1,), 1.33), 'Mo': (42, 6, (-1,), 2.16), 'Pd': (46, 10, (-1,), 2.20),
    'Ag': (47, 11, (-1,), 1.93), 'Cd': (48, 2, (-1,), 1.69), 'In': (49, 3, (3,), 1.78),
    'Sn': (50, 4, (2, 4), 1.96), 'Sb': (51, 5, (3, 5), 2.05), 'Te': (52, 6, (2, 4, 6), 2.10),
    'I': (53, 7, (1, 3, 5), 2.66), 'Yb': (70, 2, (-1,), 1.10), 'Pt': (78, 10, (-1,), 2.28),
    'Au': (79, 11, (-1,), 2.54), 'Hg': (80, 2, (-1,), 2.00), 'Tl': (81, 3, (-1,), 1.62),
    'Pb': (82, 4, (2, 4), 2.33),
}
_Z2SYM = {v[0]: k for k, v in _ELEM.items()}
_ORGANIC = ['Cl', 'Br', 'B', 'C', 'N', 'O', 'P', 'S', 'F', 'I']
_AROM_ORGANIC = {'b': 'B', 'c': 'C', 'n': 'N', 'o': 'O', 'p': 'P', 's': 'S'}
_AROM_BRACKET = {'se': 'Se', 'as': 'As', 'te': 'Te', 'b': 'B', 'c': 'C', 'n': 'N', 'o': 'O',
                 'p': 'P', 's': 'S'}
AROM = 1.5   # bond order value of an aromatic bond (RDKit getValenceContrib)


class SmilesError(ValueError):
    pass


class Mol:
    """Atoms and bonds after sanitisation (only what the features and the bigraph need)."""

    def __init__(self):
        self.sym, self.arom, self.bracket, self.hcount, self.charge = [], [], [], [], []
        self.bonds = []          # (a, b, order) order in {1, 2, 3, AROM}
        self.implicit_h = []
        self.radicals = []
        self.hyb = []
        self.bond_conj = []

    @property
    def num_atoms(self):
        return len(self.sym)

    def z(self, i):
        return _ELEM[self.sym[i]][0]

    def nbrs(self, i):
        return self._adj[i]

    def total_h(self, i):
        return self.hcount[i] + self.implicit_h[i]

    def degree(self, i):
        return len(self._adj[i])

    def _build_adj(self):
        self._adj = [[] for _ in self.sym]
        for k, (a, b, _) in enumerate(self.bonds):
            self._adj[a].append((b, k))
            self._adj[b].append((a, k))


# ----------------------------------------------------------------------------------------------
# parsing (OpenSMILES subset used by KEGG + common extras)
# ----------------------------------------------------------------------------------------------
def _parse_bracket(s, i):
    j = s.index(']', i)
    body = s[i + 1:j]
    k = 0
    while k < len(body) and body[k].isdigit():      # isotope (ignored by the features)
        k += 1
    arom = False
    if body[k] == '*':
        sym, k = '*', k + 1
    elif body[k:k + 2] in _AROM_BRACKET:
        sym, arom, k = _AROM_BRACKET[body[k:k + 2]], True, k + 2
    elif body[k] in _AROM_BRACKET:
        sym, arom, k = _AROM_BRACKET[body[k]], True, k + 1
    elif body[k:k + 2] in _ELEM and body[k + 1:k + 2].islower():
        sym, k = body[k:k + 2], k + 2
    elif body[k] in _ELEM:
        sym, k = body[k], k + 1
    else:
        raise SmilesError(f"unknown element in [{body}]")
    while k < len(body) and body[k] == '@':          # chirality (no effect on the features)
        k += 1
    h = 0
    if k < len(body) and body[k] == 'H':
        k += 1
        h = 1
        if k < len(body) and body[k].isdigit():
            h = int(body[k])
            k += 1
    chg = 0
    while k < len(body) and body[k] in '+-':
        sgn = 1 if body[k] == '+' else -1
        k += 1
        if k < len(body) and body[k].isdigit():
            n = 0
            while k < len(body) and body[k].isdigit():
                n = 10 * n + int(body[k])
                k += 1
            chg += sgn * n
        else:
            chg += sgn
    if k < len(body) and body[k] == ':':              # atom class
        k = len(body)
    if k != len(body):
        raise SmilesError(f"cannot parse bracket atom [{body}]")
    return sym, arom, h, chg, j + 1


def parse_smiles(s):
    """Atoms in input order and bonds in creation order (RDKit's bond-index order: a bond to
    the previous atom when an atom is read, a ring-closure bond when the closing digit is read)."""
    m = Mol()
    prev, branch, rings = None, [], {}
    bond_sym = None
    i = 0
    while i < len(s):
        c = s[i]
        if c == '(':
            branch.append(prev)
            i += 1
            continue
        if c == ')':
            prev = branch.pop()
            i += 1
            continue
        if c in '-=#:$/\\':
            bond_sym = c
            i += 1
            continue
        if c == '.':
            prev, bond_sym = None, None
            i += 1
            continue
        if c.isdigit() or c == '%':
            if c == '%':
                num, i = int(s[i + 1:i + 3]), i + 3
            else:
                num, i = int(c), i + 1
            if num in rings:
                a, bs = rings.pop(num)
                sym = bond_sym or bs
                m.bonds.append((a, prev, _bond_order(sym, m.arom[a], m.arom[prev])))
            else:
                rings[num] = (prev, bond_sym)
            bond_sym = None
            continue
        if c == '[':
            sym, arom, h, chg, i = _parse_bracket(s, i)
            bracket = True
        elif s[i:i + 2] in ('Cl', 'Br'):
            sym, arom, h, chg, bracket = s[i:i + 2], False, 0, 0, False
            i += 2
        elif c in _ORGANIC or c == '*':
            sym, arom, h, chg, bracket = c, False, 0, 0, c == '*'
            i += 1
        elif c in _AROM_ORGANIC:
            sym, arom, h, chg, bracket = _AROM_ORGANIC[c], True, 0, 0, False
            i += 1
        else:
            raise SmilesError(f"unexpected character {c!r} at {i} in {s}")
        idx = m.num_atoms
        m.sym.append(sym)
        m.arom.append(arom)
        m.bracket.append(bracket)
        m.hcount.append(h)
        m.charge.append(chg)
        if prev is not None:
            m.bonds.append((prev, idx, _bond_order(bond_sym, m.arom[prev], arom)))
        prev, bond_sym = idx, None
    if rings or branch:
        raise SmilesError(f"unclosed ring or branch in {s}")
    m._build_adj()
    return m


def _bond_order(sym, arom_a, arom_b):
    if sym in (None, '/', '\\'):
        return AROM if (arom_a and arom_b) else 1
    return {'-': 1, '=': 2, '#': 3, '$': 4, ':': AROM}[sym]


# ----------------------------------------------------------------------------------------------
# sanitisation (RDKit MolOps::sanitizeMol order: valence, kekulize, radicals, aromaticity,
# conjugation, hybridisation)
# ----------------------------------------------------------------------------------------------
def _valences(sym):
    return _ELEM[sym][2]


def _default_valence(sym):
    return _valences(sym)[0]


def _bond_sum(m, i, arom_as=AROM):
    return sum((arom_as if o == AROM else o) for (_, k) in m.nbrs(i) for o in [m.bonds[k][2]])


def _implicit_h(m, i):
    """RDKit Atom::calcImplicitValence for organic-subset atoms (bracket atoms: 0)."""
    sym = m.sym[i]
    if m.bracket[i] or sym == '*':
        return 0
    vals = [v for v in _valences(sym) if v >= 0]
    if not vals:
        return 0
    dv = vals[0]
    accum = _bond_sum(m, i) + m.hcount[i]
    if m.arom[i]:
        if accum > dv:               # "no H can be added": valence = largest allowed <= accum
            return 0
        ev = int(np.floor(accum + 0.1 + 0.5))
        return max(dv - ev, 0)
    ev = int(round(accum))
    for v in vals:
        if v >= ev:
            return v - ev
    return 0


def _explicit_valence(m, i):
    """Explicit valence as RDKit reports it after sanitisation (aromatic bonds 1.5, rounded;
    aromatic atoms above their default valence are clamped to an allowed valence)."""
    accum = _bond_sum(m, i) + m.hcount[i]
    sym = m.sym[i]
    vals = [v for v in _valences(sym) if v >= 0]
    if m.arom[i] and vals:
        chg = m.charge[i]
        dv = vals[0] + chg if _ELEM[sym][1] >= 4 else vals[0] - chg
        if accum > dv:
            pval = dv
            for v in vals:
                vv = v + chg if _ELEM[sym][1] >= 4 else v - chg
                if vv > accum:
                    break
                pval = vv
            return pval
    return int(np.floor(accum + 0.1 + 0.5))


def _kekulize(m):
    """Assign single/double bonds to aromatic bonds (RDKit Kekulize): atoms whose target
    valence leaves room for exactly one more bond order need a double bond; find a perfect
    matching of those atoms over aromatic bonds (most-constrained-first backtracking)."""
    arom_bonds = [k for k, b in enumerate(m.bonds) if b[2] == AROM]
    if not arom_bonds:
        return True
    need = set()
    for i in range(m.num_atoms):
        if not any(m.bonds[k][2] == AROM for (_, k) in m.nbrs(i)):
            continue
        sym = m.sym[i]
        if sym == '*':
            need.add(i)  # dummies may take a double bond if a partner needs one (resolved below)
            continue
        dv = _default_valence(sym)
        if dv < 0:
            continue
        chg = m.charge[i]
        dv = dv - chg if _ELEM[sym][1] < 4 else dv + chg  # isoelectronic target valence
        sbo = sum((1 if o == AROM else o) for (_, k) in m.nbrs(i) for o in [m.bonds[k][2]])
        sbo += m.total_h(i)
        if dv - sbo == 1:
            need.add(i)
    dummies = {i for i in need if m.sym[i] == '*'}
    adj = {i: [(j, k) for (j, k) in m.nbrs(i) if m.bonds[k][2] == AROM and j in need]
           for i in need}
    match = {}

    def solve(optional):
        free = [i for i in need if i not in match and i not in optional]
        if not free:
            return True
        # most constrained atom first
        i = min(free, key=lambda a: sum(1 for (j, _) in adj[a] if j not in match))
        for (j, k) in adj[i]:
            if j in match:
                continue
            match[i], match[j] = k, k
            if solve(optional):
                return True
            del match[i], match[j]
        return False

    ok = solve(dummies)
    for k in arom_bonds:
        a, b, _ = m.bonds[k]
        m.bonds[k] = (a, b, 2 if (match.get(a) == k and match.get(b) == k) else 1)
    return ok


def _assign_radicals(m):
    """RDKit assignRadicals: only atoms with no implicit Hs (bracket atoms)."""
    rad = [0] * m.num_atoms
    for i in range(m.num_atoms):
        sym = m.sym[i]
        if not m.bracket[i] or sym == '*' or _valences(sym) == (-1,):
            continue
        z, nouter = _ELEM[sym][0], _ELEM[sym][1]
        chg = m.charge[i]
        tv = int(round(_bond_sum(m, i))) + m.hcount[i]
        base = 2 if z <= 2 else 8
        nr = base - nouter - tv + chg
        if nr < 0:
            nr = 0
            vals = [v for v in _valences(sym) if v >= 0]
            if len(vals) > 1:
                for v in vals:
                    if v - tv + chg >= 0:
                        nr = v - tv + chg
                        break
        nr2 = nouter - tv - chg
        if nr2 >= 0:
            nr = min(nr, nr2)
        rad[i] = nr
    m.radicals = rad


def _sssr(m):
    """Minimum cycle basis (Horton): candidate cycles from BFS shortest paths, kept when
    GF(2)-independent of the shorter ones already chosen."""
    n = m.num_atoms
    nb = len(m.bonds)
    n_comp = _count_components(m)
    n_rings = nb - n + n_comp
    if n_rings <= 0:
        return []
    cands = set()
    for w in range(n):
        dist, par = {w: 0}, {w: (None, None)}
        order = [w]
        for x in order:
            for (y, k) in m.nbrs(x):
                if y not in dist:
                    dist[y], par[y] = dist[x] + 1, (x, k)
                    order.append(y)

        def path(x):
            atoms, bonds = [], []
            while x is not None:
                atoms.append(x)
                px, k = par[x]
                if k is not None:
                    bonds.append(k)
                x = px
            return atoms, bonds

        for k, (u, v, _) in enumerate(m.bonds):
            if u not in dist or v not in dist:
                continue
            au, bu = path(u)
            av, bv = path(v)
            if set(au) & set(av) != {w}:
                continue
            if k in bu or k in bv:
                continue
            mask = 0
            for kk in bu + bv + [k]:
                mask |= 1 << kk
            cands.add((len(bu) + len(bv) + 1, mask))
    basis, rings = [], []
    for size, mask in sorted(cands):
        red = mask
        for b in basis:
            red = min(red, red ^ b)
        if red:
            basis.append(red)
            basis.sort(reverse=True)
            rings.append(mask)
            if len(rings) == n_rings:
                break
    out = []
    for mask in rings:
        bonds = [k for k in range(nb) if mask >> k & 1]
        atoms = sorted({a for k in bonds for a in m.bonds[k][:2]})
        out.append((atoms, bonds))
    return out


def _count_components(m):
    seen, comps = set(), 0
    for s in range(m.num_atoms):
        if s in seen:
            continue
        comps += 1
        stack = [s]
        seen.add(s)
        while stack:
            x = stack.pop()
            for (y, _) in m.nbrs(x):
                if y not in seen:
                    seen.add(y)
                    stack.append(y)
    return comps


_VACANT, _ONE, _TWO, _ANY, _NONE = 0, 1, 2, 3, -1


def _donor_type(m, i, ring_bonds):
    """RDKit getAtomDonorTypeArom + countAtomElec + isAtomCandForArom (default model)."""
    sym = m.sym[i]
    if sym == '*':
        return _ANY
    if _ELEM[sym][0] not in (5, 6, 7, 8, 15, 16, 33, 34, 52):
        return _NONE
    dv = _default_valence(sym)
    if dv <= 1:
        return _NONE
    degree = m.degree(i) + m.total_h(i)
    if degree > 3:
        return _NONE
    orders = [(m.bonds[k][2], k, j) for (j, k) in m.nbrs(i)]
    n_mult = sum(1 for (o, _, _) in orders if o >= 2)
    if n_mult > 1:
        return _NONE
    tv = sum(o for (o, _, _) in orders) + m.total_h(i)
    if tv > dv + max(m.charge[i], 0) and _ELEM[sym][0] not in (7, 8):   # higher valence states
        return _NONE
    nlp = max(_ELEM[sym][1] - dv - m.charge[i], 0)
    nelec = (dv - degree) + nlp - m.radicals[i]
    if nelec > 1 and (tv - m.hcount[i] - m.implicit_h[i]) - m.degree(i) > 1:
        nelec = 1
    exo = [(o, j) for (o, k, j) in orders if o >= 2 and k not in ring_bonds]
    cyc_mult = any(o >= 2 and k in ring_bonds for (o, k, _) in orders)
    if nelec < 0:
        return _NONE
    if nelec == 0:
        if exo:
            return _VACANT
        return _ONE if cyc_mult else _VACANT
    if nelec == 1:
        if exo:
            j = exo[0][1]
            return _VACANT if _ELEM[m.sym[j]][3] > _ELEM[sym][3] else _ONE
        if n_mult:
            return _ONE
        return _VACANT if m.charge[i] == 1 else _NONE
    return _ONE if n_mult else _TWO


def _huckel(donors):
    lo = sum({_VACANT: 0, _ONE: 1, _TWO: 2, _ANY: 0}[d] for d in donors)
    hi = sum({_VACANT: 0, _ONE: 1, _TWO: 2, _ANY: 2}[d] for d in donors)
    if hi == 2:                     # RDKit applyHuckel: rup == 2 (3-rings) is aromatic
        return True
    return hi >= 6 and any((e - 2) % 4 == 0 for e in range(lo, hi + 1))


def _set_aromaticity(m):
    rings = _sssr(m)
    m.arom = [False] * m.num_atoms
    if not rings:
        return
    ring_bonds = {k for (_, bonds) in rings for k in bonds}
    donor = {i: _donor_type(m, i, ring_bonds) for (atoms, _) in rings for i in atoms}
    cand = [all(donor[i] != _NONE for i in atoms) for (atoms, _) in rings]
    arom_ring = [False] * len(rings)
    arom_bonds = set()

    def mark(atoms, bonds):
        for i in atoms:
            m.arom[i] = True
        arom_bonds.update(bonds)

    for r, (atoms, bonds) in enumerate(rings):
        if cand[r] and _huckel([donor[i] for i in atoms]):
            arom_ring[r] = True
            mark(atoms, bonds)
    # fused systems: pairs and triples of bond-sharing candidate rings, outer envelope
    idx = [r for r in range(len(rings)) if cand[r]]
    bsets = [set(rings[r][1]) for r in range(len(rings))]

    def envelope(rs):
        cnt = {}
        for r in rs:
            for k in rings[r][1]:
                cnt[k] = cnt.get(k, 0) + 1
        bonds = {k for k, c in cnt.items() if c == 1}
        atoms = sorted({a for r in rs for a in rings[r][0]})
        return atoms, bonds

    for a_ in range(len(idx)):
        for b_ in range(a_ + 1, len(idx)):
            ra, rb = idx[a_], idx[b_]
            if not (bsets[ra] & bsets[rb]) or (arom_ring[ra] and arom_ring[rb]):
                continue
            atoms, bonds = envelope([ra, rb])
            if _huckel([donor[i] for i in atoms]):
                arom_ring[ra] = arom_ring[rb] = True
                mark(atoms, bsets[ra] | bsets[rb])
    for a_ in range(len(idx)):
        for b_ in range(a_ + 1, len(idx)):
            for c_ in range(b_ + 1, len(idx)):
                rs = [idx[a_], idx[b_], idx[c_]]
                if all(arom_ring[r] for r in rs):
                    continue
                shared = sum(1 for x in rs for y in rs if x < y and bsets[x] & bsets[y])
                if shared < 2:
                    continue
                atoms, _ = envelope(rs)
                if _huckel([donor[i] for i in atoms]):
                    for r in rs:
                        arom_ring[r] = True
                    mark(atoms, set().union(*[bsets[r] for r in rs]))
    for k in arom_bonds:
        a, b, _ = m.bonds[k]
        m.bonds[k] = (a, b, AROM)


def _conjugation(m):
    """RDKit setConjugation: aromatic bonds, plus markConjAtomBonds over C/N/O centres."""
    conj = [o == AROM for (_, _, o) in m.bonds]

    def cand(i):
        z = _ELEM[m.sym[i]][0]
        return z <= 10 and _ELEM[m.sym[i]][1] in (4, 5, 6)

    for i in range(m.num_atoms):
        if not cand(i):
            continue
        sbo = m.degree(i) + m.total_h(i)
        if sbo < 2 or sbo > 3:
            continue
        for (_, k1) in m.nbrs(i):
            if m.bonds[k1][2] < 1.5:
                continue
            for (j, k2) in m.nbrs(i):
                if k2 == k1:
                    continue
                if m.degree(j) + m.total_h(j) > 3:
                    continue
                if cand(j):
                    conj[k1] = conj[k2] = True
    m.bond_conj = conj


def _hybridization(m):
    """RDKit setHybridization via numBondsPlusLonePairs."""
    hyb = []
    for i in range(m.num_atoms):
        sym = m.sym[i]
        z, nouter = _ELEM[sym][0], _ELEM[sym][1]
        if z == 0:
            hyb.append(HYB_UNSPEC)
            continue
        deg = m.degree(i) + m.total_h(i)
        if z <= 1:
            norbs = deg
        else:
            tv = _explicit_valence(m, i) + m.implicit_h[i]
            chg = m.charge[i]
            free = nouter - (tv + chg)
            if tv + nouter - chg < 8:
                norbs = deg + (free - m.radicals[i]) // 2 + m.radicals[i]
            else:
                norbs = deg + free // 2
        if norbs <= 1:
            h = HYB_S
        elif norbs == 2:
            h = HYB_SP
        elif norbs == 3:
            h = HYB_SP2
        elif norbs == 4:
            has_conj = any(m.bond_conj[k] for (_, k) in m.nbrs(i))
            h = HYB_SP2 if (deg <= 3 and has_conj) else HYB_SP3
        elif norbs == 5:
            h = HYB_SP3D
        elif norbs == 6:
            h = HYB_SP3D2
        else:
            h = HYB_UNSPEC
        hyb.append(h)
    m.hyb = hyb


def _remove_hs(m):
    """RDKit RemoveHs for plain neutral [H] atoms bonded to one heavy atom: the H becomes an
    explicit H count on its neighbour."""
    drop = [i for i in range(m.num_atoms) if m.sym[i] == 'H' and m.charge[i] == 0
            and m.hcount[i] == 0 and m.degree(i) == 1 and m.sym[m.nbrs(i)[0][0]] != 'H']
    if not drop:
        return m
    dset = set(drop)
    for i in drop:
        j = m.nbrs(i)[0][0]
        m.hcount[j] += 1
    keep = [i for i in range(m.num_atoms) if i not in dset]
    remap = {o: n for n, o in enumerate(keep)}
    out = Mol()
    for name in ('sym', 'arom', 'bracket', 'hcount', 'charge'):
        setattr(out, name, [getattr(m, name)[i] for i in keep])
    out.bonds = [(remap[a], remap[b], o) for (a, b, o) in m.bonds if a in remap and b in remap]
    out._build_adj()
    return out


def mol_from_smiles(smiles):
    """Chem.MolFromSmiles (dataset.py:33): parse + sanitise.  Raises SmilesError where RDKit
    would return None (unparsable input, failed kekulisation)."""
    m = _remove_hs(parse_smiles(smiles))
    m.implicit_h = [0] * m.num_atoms
    m.implicit_h = [_implicit_h(m, i) for i in range(m.num_atoms)]
    # explicit-H organic atoms (from removed [H]) keep implicit H = default - valence
    if not _kekulize(m):
        raise SmilesError(f"cannot kekulize {smiles}")
    _assign_radicals(m)
    _set_aromaticity(m)
    _conjugation(m)
    _hybridization(m)
    return m


def atom_features(m):
    """CanonicalAtomFeaturizer('h') (dataset.py:23) -> float32[n, 74]."""
    n = m.num_atoms
    f = np.zeros((n, FEAT_SIZE), dtype=np.float32)
    for i in range(n):
        sym = m.sym[i]
        if sym in ATOM_TYPES:
            f[i, ATOM_TYPES.index(sym)] = 1
        d = m.degree(i)
        if d <= 10:
            f[i, 43 + d] = 1
        iv = m.implicit_h[i]
        if iv <= 6:
            f[i, 54 + iv] = 1
        f[i, 61] = m.charge[i]
        f[i, 62] = m.radicals[i]
        if m.hyb[i] in (HYB_SP, HYB_SP2, HYB_SP3, HYB_SP3D, HYB_SP3D2):
            f[i, 63 + m.hyb[i]] = 1
        f[i, 68] = 1.0 if m.arom[i] else 0.0
        th = m.total_h(i)
        if th <= 4:
            f[i, 69 + th] = 1
    return f


def canonical_ranks(m):
    """Chem.CanonicalRankAtoms (RDKit's canonicalisation, Schneider, Sayle & Landrum, J. Chem. Inf.
    Model. 2015, restated; parity with RDKit unpinned): atoms are partitioned by the base
    invariants RDKit compares first (degree, atomic number, isotope, total H, formal charge);
    partitions are refined by each atom's sorted (neighbour rank, bond order) list until stable;
    a partition still tied after refinement (symmetry) is split by giving its lowest-index atom
    the lower rank, then refinement resumes.  Returns rank[old atom] in 0 .. n-1."""
    n = m.num_atoms
    if n == 0:
        return []
    code = {1: 1, 2: 2, 3: 3, AROM: 12}

    def dense(keys):
        order = sorted(range(n), key=lambda i: (keys[i], i))
        rk, r = [0] * n, 0
        for t, i in enumerate(order):
            if t and keys[i] != keys[order[t - 1]]:
                r = t
            rk[i] = r
        return rk

    ranks = dense([(m.degree(i), m.z(i), 0, m.total_h(i), m.charge[i]) for i in range(n)])
    while True:
        while True:  # refine by neighbourhoods
            keys = [(ranks[i], tuple(sorted((ranks[j], code[m.bonds[k][2]]) for (j, k) in m.nbrs(i))))
                    for i in range(n)]
            new = dense(keys)
            if len(set(new)) == len(set(ranks)):
                ranks = new
                break
            ranks = new
        if len(set(ranks)) == n:
            return ranks
        # break the first tie: the lowest-index atom of the lowest tied rank goes first
        tied = min(r for r in set(ranks) if ranks.count(r) > 1)
        first = min(i for i in range(n) if ranks[i] == tied)
        ranks = dense([(ranks[i], 0 if i == first else 1) for i in range(n)])


def smiles_to_bigraph(smiles, add_self_loop=True, canonical_atom_order=True):
    """mol_to_bigraph(Chem.MolFromSmiles(s), add_self_loop=True,
    node_featurizer=CanonicalAtomFeaturizer('h')) (dataset.py:33-35): a MolGraph whose edges
    are (u_i->v_i),(v_i->u_i) per bond in bond order, then self-loops; ndata['h'] f32[n,74].
    canonical_atom_order (dgllife's default, True): the atoms renumbered as dgllife does,
    ``RenumberAtoms(mol, CanonicalRankAtoms(mol))`` — new atom k is old atom rank[k] — with the
    bonds in their original order and orientation (RDKit RenumberAtoms)."""
    from .batching import bigraph_from_bonds
    m = mol_from_smiles(smiles)
    feats = atom_features(m)
    bonds = np.array([(a, b) for (a, b, _) in m.bonds], dtype=np.int32).reshape(-1, 2)
    if canonical_atom_order and m.num_atoms:
        new_order = np.asarray(canonical_ranks(m), dtype=np.int64)  # new atom k <- old new_order[k]
        inv = np.empty_like(new_order)
        inv[new_order] = np.arange(len(new_order))
        feats = feats[new_order]
        bonds = inv[bonds].astype(np.int32).reshape(-1, 2)
    return bigraph_from_bonds(m.num_atoms, bonds, feats, add_self_loop=add_self_loop)


class MolDataSet:
    """Graph-view part of dataset.py:16-49 ``MolDataSet``: rows of a (smiles, label) CSV;
    ``ds[i]`` -> (MolGraph with ndata['h'], multi-hot label f32[num_classes]).  Labels are
    the comma-separated class ids one-hot-summed as in dataset.py:29-31.  Graphs are built
    once and cached (the reference re-runs RDKit every epoch)."""

    def __init__(self, data_path, labels_split=',', num_classes=11):
        import csv
        with open(data_path, newline="") as f:
            rows = list(csv.DictReader(f))
        self.smiles = [r["smiles"] for r in rows]
        self.labels = [r["label"] for r in rows]
        self.labels_split = labels_split
        self.num_classes = num_classes
        self._cache = {}

    def __len__(self):
        return len(self.smiles)

    def __getitem__(self, index):
        if index not in self._cache:
            y = np.zeros(self.num_classes, dtype=np.float32)
            for c in self.labels[index].split(self.labels_split):
                y[int(c)] += 1
            self._cache[index] = (smiles_to_bigraph(self.smiles[index]), y)
        return self._cache[index]


def collate(samples, group_size=None):
    """dataset.py:51-57 for the graph view: dgl.batch of the graphs + stacked labels."""
    import torch
    from .batching import batch
    graphs, labels = zip(*samples)
    return batch(graphs, group_size=group_size), torch.as_tensor(np.stack(labels))
