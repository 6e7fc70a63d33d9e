#!/usr/bin/env python3
"""Derive H3 v3.7's base-cell neighbour tables and the aperture-7 digit-walk tables.

H3's ``kRing`` / ``hexRing`` (reached from ``H3IndexSystem.kRing`` / ``kLoop``,
reference ``H3IndexSystem.scala:182-205``, dependency ``com.uber:h3:3.7.0`` -- not
vendored) walk from cell to cell with ``h3NeighborRotations``, which needs:

* ``baseCellNeighbors[122][7]`` / ``baseCellNeighbor60CCWRots[122][7]``: the base cell
  one step away in each of the 7 IJK directions (0 = itself; a pentagon's K
  direction is deleted = 127) and the ccw 60-degree rotations from the source's
  frame into the neighbour's.  Derived here: the step is taken in the source's home
  face IJK frame; while it stays on the face the neighbour and rotation are
  ``faceIjkBaseCells`` entries (tools/gen_h3_tables.py, checked against published
  entries); past the face edge (overage) the neighbour is the base cell nearest to
  the stepped position on the sphere, and the rotation is read, as for
  ``faceIjkBaseCells``, from the azimuth of the two frames' i-axes at the neighbour's
  centre.  Every overage rotation must round cleanly to a multiple of 60 degrees.
* ``NEW_DIGIT_II / NEW_ADJUSTMENT_II / NEW_DIGIT_III / NEW_ADJUSTMENT_III[7][7]``:
  the child digit after a unit step from child digit ``d`` in direction ``dir`` and
  the step carried to the parent.  Derived from IJK arithmetic: child centre =
  unit(d) + unit(dir) in the child grid, decomposed as parent step * aperture-7
  (ccw for Class II children, cw for Class III) + child digit.

Checks: H3's published rows for base cells 0-4 (below) and mutual adjacency
(``b`` is a neighbour of each of its neighbours).  Output: ``h3_neighbors.inc`` in
``mosaic_amd/csrc`` (product) and ``oracle`` (oracle), byte-identical data.
"""
import math
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import gen_h3_tables as T  # noqa: E402

UNIT = [(0, 0, 0), (0, 0, 1), (0, 1, 0), (0, 1, 1), (1, 0, 0), (1, 0, 1), (1, 1, 0)]
INVALID = 127

# rows of H3 v3 baseCells.c as published, used only as checks of the derivation
PUBLISHED_NEIGHBORS = {
    0: ([0, 1, 5, 2, 4, 3, 8], [0, 5, 0, 0, 1, 5, 1]),
    1: ([1, 7, 6, 9, 0, 3, 2], [0, 0, 1, 0, 1, 0, 1]),
    2: ([2, 6, 10, 11, 0, 1, 5], [0, 0, 0, 0, 0, 5, 0]),
    3: ([3, 13, 1, 7, 4, 12, 0], [0, 5, 0, 0, 2, 5, 1]),
    4: ([4, INVALID, 15, 8, 3, 0, 12], [0, -1, 1, 0, 3, 4, 2]),
}


def digit_of(ijk):
    n = T.norm_ijk(*ijk)
    return UNIT.index(n) if n in UNIT else None


def add(a, b):
    return (a[0] + b[0], a[1] + b[1], a[2] + b[2])


def down_ap7(ijk, cw):
    """IJK in the parent grid -> the same point in the child (aperture-7) grid."""
    i, j, k = ijk
    if not cw:  # _downAp7: i -> (3,0,1), j -> (1,3,0), k -> (0,1,3)
        iv, jv, kv = (3, 0, 1), (1, 3, 0), (0, 1, 3)
    else:  # _downAp7r
        iv, jv, kv = (3, 1, 0), (0, 3, 1), (1, 0, 3)
    return T.norm_ijk(i * iv[0] + j * jv[0] + k * kv[0], i * iv[1] + j * jv[1] + k * kv[1],
                      i * iv[2] + j * jv[2] + k * kv[2])


def digit_tables(cw):
    """NEW_DIGIT / NEW_ADJUSTMENT: child position unit(d) + unit(dir) = down(parent step)
    + unit(d').  H3 descends to a Class III resolution with _downAp7 (ccw; the _II tables,
    used when the child resolution is Class III) and to Class II with _downAp7r (cw;
    the _III tables)."""
    nd = [[0] * 7 for _ in range(7)]
    na = [[0] * 7 for _ in range(7)]
    for d in range(7):
        for s in range(7):
            p = T.norm_ijk(*add(UNIT[d], UNIT[s]))
            hit = None
            for a in range(7):
                base = down_ap7(UNIT[a], cw=cw)
                for c in range(7):
                    if T.norm_ijk(*add(base, UNIT[c])) == p:
                        assert hit is None or hit == (a, c), ("ambiguous decomposition", d, s)
                        hit = (a, c)
            assert hit is not None, ("no decomposition", d, s)
            na[d][s], nd[d][s] = hit
    return nd, na


# hex2d angle of each direction's unit vector (I = 0, ccw)
THETA = {1: 240.0, 2: 120.0, 3: 180.0, 4: 0.0, 5: 300.0, 6: 60.0}


def frame_rotation(b, d, n, home, cen):
    """ccw 60-degree rotations taking directions in b's frame to n's frame, read off the
    ray between the centres: leaving b along direction d (angle THETA[d]) it must arrive
    in n's home-face hex2d frame pointing back at b from angle THETA[d] + 180 + 60 rot.
    Exact for hexagon targets (it reproduces all 659 in-face faceIjkBaseCells entries);
    a pentagon target's frame is cut (its deleted K sector), so the fraction is
    rounded down -- the rule that reproduces all 25 in-face hexagon -> pentagon
    entries."""
    hf, hijk = home[n]
    _, blat, blon = cen[b]
    x, y = T.geo_to_hex2d_res0(blat, blon, hf)
    cx, cy = T.ijk_to_hex2d(*hijk)
    phi = math.degrees(math.atan2(y - cy, x - cx))
    q = (phi - THETA[d] - 180.0) / 60.0
    q -= 6.0 * math.floor(q / 6.0)
    if n in T.PENTAGONS:
        r = math.floor(q + 1e-9)
        return int(r) % 6, 0.0
    r = round(q)
    return int(r) % 6, abs(q - r)


def shared_face_rotation(b, n, bc_of, rot):
    """Rotation from hexagon b's frame into pentagon n's frame read off a face g that
    holds both: faceIjkBaseCells gives g -> b and g -> n, so b -> n = rot(g->n) -
    rot(g->b).  A pentagon's frame is cut, so the measurement must come from the
    faceIjkBaseCells convention, not from geometry; every shared face must agree."""
    vals = set()
    for (g, i, j, k), c in bc_of.items():
        if c != n:
            continue
        for (g2, i2, j2, k2), c2 in bc_of.items():
            if g2 == g and c2 == b:
                vals.add((rot[(g, i, j, k)] - rot[(g2, i2, j2, k2)]) % 6)
    assert len(vals) == 1, ("hexagon -> pentagon rotation ambiguous", b, n, vals)
    return vals.pop()


def pentagon_labels(b, home, bc_of, cen):
    """The five neighbours of pentagon b by direction.  Its IJK frame has the K sector
    deleted, so going ccw (seen from outside) round b the neighbours take the labels
    J, JK, (K deleted), IK, I, IJ; J is the in-face step from the home face."""
    f, ijk = home[b]
    v = cen[b][0]
    dist = sorted((float(np.linalg.norm(cen[c][0] - v)), c) for c in range(122) if c != b)
    assert dist[4][0] < 0.8 * dist[5][0], ("pentagon neighbours not separated", b)
    nbrs = [c for _, c in dist[:5]]
    e1 = np.cross([0.0, 0.0, 1.0], v)
    if np.linalg.norm(e1) < 1e-6:
        e1 = np.cross([1.0, 0.0, 0.0], v)
    e1 /= np.linalg.norm(e1)
    e2 = np.cross(v, e1)
    ang = {c: math.atan2(float(np.dot(cen[c][0], e2)), float(np.dot(cen[c][0], e1))) for c in nbrs}
    ccw = sorted(nbrs, key=lambda c: ang[c])
    j_n = bc_of[(f,) + T.norm_ijk(*add(ijk, UNIT[2]))]
    jk_n = bc_of[(f,) + T.norm_ijk(*add(ijk, UNIT[3]))]
    s = ccw.index(j_n)
    ccw = ccw[s:] + ccw[:s]
    lab = dict(zip((2, 3, 5, 4, 6), ccw))
    assert lab[3] == jk_n, ("pentagon JK neighbour is not next ccw after J", b)
    return lab


def neighbors(home, bc_of, rot, cen):
    nb = [[0] * 7 for _ in range(122)]
    nr = [[0] * 7 for _ in range(122)]
    worst = 0.0
    for b in range(122):
        f, ijk = home[b]
        nb[b][0], nr[b][0] = b, 0
        lab = pentagon_labels(b, home, bc_of, cen) if b in T.PENTAGONS else None
        for d in range(1, 7):
            if lab is not None and d == 1:
                nb[b][d], nr[b][d] = INVALID, -1
                continue
            pos = T.norm_ijk(*add(ijk, UNIT[d]))
            if max(pos) <= 2:
                key = (f,) + pos
                n = bc_of[key]
                if lab is not None:
                    assert lab[d] == n, ("pentagon label disagrees with the in-face step", b, d)
                if n not in T.PENTAGONS:
                    r, res = frame_rotation(b, d, n, home, cen)
                    assert r == rot[key], ("frame rotation disagrees with faceIjkBaseCells", b, d, n, r, rot[key])
                nb[b][d], nr[b][d] = n, rot[key]
                continue
            if lab is not None:
                n = lab[d]
            else:
                x, y = T.ijk_to_hex2d(*pos)
                lat, lon = T.hex2d_to_geo_res0(x, y, f)
                v = T.geo_to_vec(lat, lon)
                dist = sorted((float(np.linalg.norm(cen[c][0] - v)), c) for c in range(122))
                assert dist[0][0] < 0.5 * dist[1][0], ("ambiguous overage neighbour", b, d)
                n = dist[0][1]
            if n in T.PENTAGONS and lab is None:
                r = shared_face_rotation(b, n, bc_of, rot)
            else:
                r, res = frame_rotation(b, d, n, home, cen)
                worst = max(worst, res)
            nb[b][d], nr[b][d] = n, r
    return nb, nr, worst


def build():
    home, bc_of, rot, cen = T.build()
    nb, nr, worst = neighbors(home, bc_of, rot, cen)
    print("overage rotations: worst distance from a multiple of 60 deg = %.3f (x 60 deg)" % worst)
    bad = 0
    for b, (en, er) in PUBLISHED_NEIGHBORS.items():
        if nb[b] != en or nr[b] != er:
            bad += 1
            print("published-row mismatch", b, "derived", nb[b], nr[b], "published", en, er)
    # mutual adjacency
    for b in range(122):
        for d in range(1, 7):
            n = nb[b][d]
            if n == INVALID:
                continue
            if b not in nb[n][1:]:
                bad += 1
                print("not mutual", b, d, n)
    assert worst < 0.25 and bad == 0, "neighbour derivation failed its checks"
    dig2, adj2 = digit_tables(cw=False)
    dig3, adj3 = digit_tables(cw=True)
    return nb, nr, (dig2, adj2, dig3, adj3)


def emit(path, nb, nr, dt):
    L = ["/* Generated by tools/gen_h3_neighbors.py -- H3 v3.7 base-cell neighbours and digit-walk",
         "   tables (data restated for com.uber:h3:3.7.0, see the generator's docstring). */",
         "#ifndef H3T_QUAL", "#define H3T_QUAL static const", "#endif",
         "#define H3T_INVALID_BASE_CELL 127",
         "/* baseCellNeighbors[base cell][direction] */",
         "H3T_QUAL unsigned char H3T_BASE_CELL_NEIGHBORS[122][7] = {"]
    for b in range(122):
        L.append("    {%s}," % ", ".join(str(v) for v in nb[b]))
    L.append("};")
    L.append("/* baseCellNeighbor60CCWRots[base cell][direction] (-1: deleted direction) */")
    L.append("H3T_QUAL signed char H3T_BASE_CELL_NEIGHBOR_ROTS[122][7] = {")
    for b in range(122):
        L.append("    {%s}," % ", ".join(str(v) for v in nr[b]))
    L.append("};")
    for name, t in zip(("H3T_NEW_DIGIT_II", "H3T_NEW_ADJUSTMENT_II", "H3T_NEW_DIGIT_III", "H3T_NEW_ADJUSTMENT_III"), dt):
        L.append("H3T_QUAL unsigned char %s[7][7] = {" % name)
        for row in t:
            L.append("    {%s}," % ", ".join(str(v) for v in row))
        L.append("};")
    with open(path, "w") as fh:
        fh.write("\n".join(L) + "\n")


def main():
    nb, nr, dt = build()
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    for rel in ("mosaic_amd/csrc/h3_neighbors.inc", "oracle/h3_neighbors.inc"):
        emit(os.path.join(root, rel), nb, nr, dt)
        print("wrote", rel)


if __name__ == "__main__":
    main()
