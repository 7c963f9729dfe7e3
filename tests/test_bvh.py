"""Triangle BVH (csrc/bvh.cpp) on the CPU: structure, and the bound the exact
traversal rests on.

The reference's closest hit is brute force over every triangle with first-
index ties (scene_basics.h:426-459 under bvh.h:55-77's single leaf).  The
BVH returns the same hit iff no box ever excludes a triangle that the fp32
test accepts.  These tests take the accepting t of EVERY triangle from the
oracle's own test (oro_hit_each) on adversarial rays -- at vertices, along
edges, grazing planes -- and check that the exact ray point at that t lies
inside every box on the triangle's path to the root, with margin for the
traversal's slab rounding; then a float32 emulation of the device traversal
reproduces the oracle's closest hit.  The device traversal itself is checked
against the brute-force loop bit-for-bit in tests/test_gpu.py.
"""
import numpy as np
import pytest

from conftest import CORNELL, CUBE_OBJ, SCENE0, SPHERE_OBJ, product_scene

SPHERE_SCENE = CORNELL + [((0.3, -1.2, 4.2), (0.0, 0.4, 0.0), (1.2, 1.2, 1.2), SPHERE_OBJ, "*Kd 0.2 0.6 0.3*")]
CLUTTER_SCENE = SPHERE_SCENE + [
    ((-0.9, -1.4, 3.9), (0.2, 0.7, 0.1), (0.7, 0.7, 0.7), CUBE_OBJ, "*Kd 0.5 0.5 0.5*"),
    ((0.8, 0.9, 4.6), (0.0, 0.0, 0.5), (0.5, 0.5, 0.5), SPHERE_OBJ, "*Kd 0.9 0.1 0.1*"),
]


def _tree(nodes):
    """parent links: leaf pair ranges and node parents from the export."""
    kids = np.ascontiguousarray(nodes[:, 12:14]).view(np.int32)
    parent = {0: None}
    leaves = []  # (first_pair, n_pairs, parent node, child slot)
    for n in range(len(nodes)):
        for c in range(2):
            k = int(kids[n, c])
            if k >= 0:
                parent[k] = (n, c)
            else:
                code = ~k
                leaves.append((code >> 4, (code & 15) + 1, n, c))
    return kids, parent, leaves


def _box(nodes, n, c):
    q = nodes[n, 6 * c:6 * c + 6].astype(np.float64)
    return q[0::2], q[1::2]  # lo xyz, hi xyz


@pytest.fixture(scope="module")
def sphere_scene(oracle):
    return product_scene(SPHERE_SCENE, device=False), oracle.OracleScene(SPHERE_SCENE)


def test_bvh_selected_by_size():
    small = product_scene(SCENE0, device=False).bvh_info()
    assert small["accel"] == "brute"  # 30 triangles: the packed brute-force loop
    big = product_scene(SPHERE_SCENE, device=False).bvh_info()
    assert big["has_bvh"] and big["accel"] == "bvh" and big["status"] == "ok"
    assert 1 <= big["depth"] <= 32


@pytest.mark.parametrize("recs", [SPHERE_SCENE, CLUTTER_SCENE], ids=["sphere", "clutter"])
def test_bvh_structure(recs):
    P = product_scene(recs, device=False)
    nodes, pairs, big = P.export_bvh()
    kids, parent, leaves = _tree(nodes)
    idx = np.ascontiguousarray(pairs[:, 36:38]).view(np.int32)
    # the Cornell walls and light (18 large triangles) are in the brute-force
    # pre-pass (with the clutter's cube faces: bvh.cpp kBigFrac), ascending
    bigr = big[big != 0x7FFFFFFF]
    assert set(range(18)) <= set(bigr.tolist()) and len(bigr) <= 32 and np.all(np.diff(bigr) > 0)
    # breadth-first numbering: children come after their parent
    for n in range(len(nodes)):
        for c in range(2):
            if kids[n, c] >= 0:
                assert kids[n, c] > n
    assert len(parent) == len(nodes)  # every node reachable from the root
    # leaves tile the pair array; each triangle appears exactly once
    covered = np.zeros(len(pairs), int)
    for first, npairs, _, _ in leaves:
        covered[first:first + npairs] += 1
    assert np.all(covered == 1)
    real = idx[idx != 0x7FFFFFFF]
    assert sorted(real.tolist() + bigr.tolist()) == list(range(P.nT))
    pad = idx == 0x7FFFFFFF
    assert np.all(pairs[:, :36].reshape(-1, 18, 2)[pad.nonzero()[0], :, pad.nonzero()[1]] == 0)
    # a child's box lies inside the box its parent stores for it
    for n in range(1, len(nodes)):
        pn, pc = parent[n]
        plo, phi = _box(nodes, pn, pc)
        for c in range(2):
            lo, hi = _box(nodes, n, c)
            assert np.all(lo >= plo) and np.all(hi <= phi)


def _adversarial_rays(tris, cam_origin, rng, n):
    """Origins: the camera, points on triangles, points in the scene box.
    Targets: vertices, edge points (just inside / on / just outside), centres,
    and directions nearly parallel to a triangle's plane."""
    v = tris[:, 0:9].reshape(-1, 3, 3).astype(np.float64)
    nrm = tris[:, 18:21].astype(np.float64)
    lo, hi = v.reshape(-1, 3).min(0), v.reshape(-1, 3).max(0)
    nT = len(tris)
    O, D = [], []
    for k in range(n):
        kind = k % 4
        if kind == 0:
            o = cam_origin
        elif kind == 1:
            i = rng.randint(nT)
            a, b = rng.uniform(0, 1, 2)
            if a + b > 1:
                a, b = 1 - a, 1 - b
            o = v[i, 0] + a * (v[i, 1] - v[i, 0]) + b * (v[i, 2] - v[i, 0])
        else:
            o = rng.uniform(lo, hi)
        i = rng.randint(nT)
        sel = rng.randint(5)
        if sel == 0:
            tgt = v[i, rng.randint(3)]
        elif sel in (1, 2):
            j = rng.randint(3)
            s = rng.uniform(0, 1)
            tgt = v[i, j] + s * (v[i, (j + 1) % 3] - v[i, j])
            ctr = v[i].mean(0)
            tgt = tgt + (tgt - ctr) * rng.choice([-1e-6, 0.0, 1e-6, 1e-7])
        elif sel == 3:
            tgt = v[i].mean(0)
        else:  # grazing: direction almost in triangle i's plane
            n_ = nrm[i] / max(np.linalg.norm(nrm[i]), 1e-30)
            tgt = v[i].mean(0) + rng.uniform(-1, 1, 3) * 0.3
            o = tgt - 2.0 * np.cross(n_, rng.normal(size=3))
            d = tgt - o
            d = d / np.linalg.norm(d)
            d = d - np.dot(d, n_) * n_ * (1 - rng.uniform(1.0001e-4, 3e-4) / max(abs(np.dot(d, n_)), 1e-30))
            O.append(o)
            D.append(d / np.linalg.norm(d))
            continue
        d = tgt - o
        nd = np.linalg.norm(d)
        if nd < 1e-6:
            d, nd = rng.normal(size=3), 1.0
        O.append(o)
        D.append(d / np.linalg.norm(d))
    return np.asarray(O, np.float32), np.asarray(D, np.float32)


def _r_all(tris, cam_origin):
    v = np.abs(tris[:, 0:9]).max()
    return float(max(v, np.abs(cam_origin).max()) + 1.0)


@pytest.mark.parametrize("recs", [SPHERE_SCENE, CLUTTER_SCENE], ids=["sphere", "clutter"])
def test_acceptance_inside_every_ancestor_box(oracle, recs):
    P, Q = product_scene(recs, device=False), oracle.OracleScene(recs)
    tris = P.triangles()
    cam = P.camera()
    cam_origin = cam[:3, 3].astype(np.float64)
    nodes, pairs, big = P.export_bvh()
    _, parent, leaves = _tree(nodes)
    bigset = set(big.tolist())
    idx = np.ascontiguousarray(pairs[:, 36:38]).view(np.int32)
    tri_slot = {}
    for first, npairs, pn, pc in leaves:
        for j in range(first, first + npairs):
            for h in range(2):
                if idx[j, h] != 0x7FFFFFFF:
                    tri_slot[int(idx[j, h])] = (pn, pc)
    margin = 2.0 ** -18 * _r_all(tris, cam_origin)  # > the slab test's plane displacement (6uR)
    rng = np.random.RandomState(11)
    O, D = _adversarial_rays(tris, cam_origin, rng, 3000)
    accepted = 0
    for o, d in zip(O, D):
        t = Q.hit_each(o, d)
        for i in np.nonzero(~np.isnan(t))[0]:
            accepted += 1
            x = o.astype(np.float64) + float(t[i]) * d.astype(np.float64)
            if int(i) in bigset:
                continue  # tested by the brute-force pre-pass for every ray
            slot = tri_slot[int(i)]
            while slot is not None:
                lo, hi = _box(nodes, *slot)
                assert np.all(x >= lo + margin) and np.all(x <= hi - margin), (i, slot, x, lo, hi)
                slot = parent[slot[0]]
    assert accepted > 1000


def _traverse(nodes, pairs, big, kids, o, d, oracle_scene):
    """float32 emulation of ipt_device.h::closest_hit_bvh (exact reciprocal
    instead of v_rcp_f32; the leaf test's t from the oracle's own test)."""
    f = np.float32
    o32, d32 = o.astype(f), d.astype(f)
    with np.errstate(divide="ignore", invalid="ignore", over="ignore"):
        inv = np.where(np.abs(d32) < f(2.0 ** -60), f(0), f(1) / d32).astype(f)
        off = np.where(np.abs(d32) < f(2.0 ** -60), f(np.nan), -(o32 * inv)).astype(f)
    teach = oracle_scene.hit_each(o, d)
    idx = np.ascontiguousarray(pairs[:, 36:38]).view(np.int32)
    bt, bi = np.float32(np.inf), -1
    for i in big:  # the pre-pass over the large triangles
        if i != 0x7FFFFFFF and not np.isnan(teach[i]) and (teach[i] < bt or (teach[i] == bt and i < bi)):
            bt, bi = teach[i], int(i)
    stack, node = [], 0
    while node is not None:
        while node is not None and node >= 0:
            q = nodes[node]
            hit, en = [], []
            for c in range(2):
                b = q[6 * c:6 * c + 6]
                with np.errstate(invalid="ignore", over="ignore"):
                    t0 = (b[0::2].astype(np.float64) * inv + off).astype(f)  # one rounding, like the fma
                    t1 = (b[1::2].astype(np.float64) * inv + off).astype(f)
                mn, mx = np.fmin(t0, t1), np.fmax(t0, t1)
                e = max(np.nanmax(np.append(mn, 0.0)), 0.0)
                x = min(np.nanmin(np.append(mx, np.inf)), bt)
                hit.append(e <= x)
                en.append(e)
            c0, c1 = int(np.int32(q[12:13].view(np.int32)[0])), int(q[13:14].view(np.int32)[0])
            if hit[0] and hit[1]:
                near, far = (c0, c1) if en[0] <= en[1] else (c1, c0)
                stack.append(far)
                node = near
            elif hit[0] or hit[1]:
                node = c0 if hit[0] else c1
            else:
                node = stack.pop() if stack else None
        if node is not None:
            code = ~node
            first, npairs = code >> 4, (code & 15) + 1
            for j in range(first, first + npairs):
                for h in range(2):
                    i = int(idx[j, h])
                    if i == 0x7FFFFFFF or np.isnan(teach[i]):
                        continue
                    t = teach[i]
                    if t < bt or (t == bt and i < bi):
                        bt, bi = t, i
            node = stack.pop() if stack else None
    return bt, bi


def test_emulated_traversal_matches_oracle_closest_hit(sphere_scene):
    P, Q = sphere_scene
    nodes, pairs, big = P.export_bvh()
    kids, _, _ = _tree(nodes)
    tris = P.triangles()
    cam_origin = P.camera()[:3, 3].astype(np.float64)
    O, D = _adversarial_rays(tris, cam_origin, np.random.RandomState(5), 400)
    t_ref, i_ref = Q.closest_hit(O, D)
    for k in range(len(O)):
        bt, bi = _traverse(nodes, pairs, big, kids, O[k], D[k], Q)
        assert bi == i_ref[k], k
        if bi >= 0:
            assert np.float32(bt).view(np.uint32) == t_ref[k].view(np.uint32)


def test_never_hit_triangle_left_out(tmp_path):
    """A degenerate triangle (collinear vertices: zero face normal, so |n.d| =
    0 < 1e-4 rejects every ray) is left out of the tree; the rest still gets
    a BVH."""
    p = tmp_path / "deg.obj"
    p.write_text("v 0 0 4\nv 1 0 4\nv 2 0 4\nf 1 2 3\n")
    recs = SPHERE_SCENE + [((0, 0, 0), (0, 0, 0), (1, 1, 1), str(p), "*Kd 0.5 0.5 0.5*")]
    P = product_scene(recs, device=False)
    assert P.nT == 1299 and np.all(P.triangles()[1298, 18:21] == 0)
    info = P.bvh_info()
    assert info["has_bvh"] and info["accel"] == "bvh"
    _, pairs, big = P.export_bvh()
    idx = np.ascontiguousarray(pairs[:, 36:38]).view(np.int32)
    got = idx[idx != 0x7FFFFFFF].tolist() + big[big != 0x7FFFFFFF].tolist()
    assert 1298 not in got and sorted(got) == list(range(1298))


@pytest.mark.parametrize("name", ["sphere", "clutter", "northstar"])
def test_wide_nodes_nest_and_order_children(name):
    """WideNode (scene_layout.h, bvh.cpp build_wide): every inner child's own
    children lie inside the box its parent slot stores, and each slot's pad
    word gives the 8 children's ranks in the octant front-to-back order (a
    permutation; the cooperative traversal's lane j reads child j's rank)."""
    from conftest import NORTHSTAR

    recs = {"sphere": SPHERE_SCENE, "clutter": CLUTTER_SCENE, "northstar": NORTHSTAR}[name]
    P = product_scene(recs, device=False)
    wide = P.export_wide()
    assert len(wide) == P.bvh_info()["wide_nodes"] > 0
    if name == "northstar":
        assert len(wide) * 256 <= 32 * 1024  # the sphere-only tree (cube in the pre-pass) fits the LDS stage
    refs = wide[:, :, 6].copy().view(np.int32)
    used = refs != np.int32(-2 ** 31)
    for n in range(len(wide)):
        for k in np.nonzero(used[n] & (refs[n] >= 0))[0]:
            c = refs[n, k]
            cu = used[c]
            assert np.all(wide[c, cu, 0:3] >= wide[n, k, 0:3]) and np.all(wide[c, cu, 3:6] <= wide[n, k, 3:6])
        for o in range(8):
            perm = int(wide[n, o, 7:8].copy().view(np.uint32)[0])
            assert sorted((perm >> (3 * r)) & 7 for r in range(8)) == list(range(8))


def _shadow_rays(tris, n, rng, edge_frac=0.3):
    """Shadow rays as the megakernel builds them: origin on a random source
    triangle, target point on a random emitter (near its edges and corners
    for edge_frac of them); returns O, D, targets, sources, emitter index."""
    emit = np.nonzero(tris[:, 56] >= 0)[0]
    v = tris[:, 0:9].reshape(-1, 3, 3).astype(np.float64)

    def on_tri(idx, a, b):
        flip = a + b > 1
        a, b = np.where(flip, 1 - a, a), np.where(flip, 1 - b, b)
        return v[idx, 0] + a[:, None] * (v[idx, 1] - v[idx, 0]) + b[:, None] * (v[idx, 2] - v[idx, 0])

    src = rng.randint(0, len(tris), n)
    O = on_tri(src, *rng.uniform(0, 1, (2, n)))
    e = rng.randint(0, len(emit), n)
    ab = rng.uniform(0, 1, (2, n))
    edge = rng.uniform(0, 1, n) < edge_frac
    ab[:, edge] = np.round(ab[:, edge] * 4) / 4 + rng.normal(0, 1e-6, (2, int(edge.sum())))
    pt = on_tri(emit[e], np.clip(ab[0], 0, 1), np.clip(ab[1], 0, 1))
    D = pt - O
    dist = np.linalg.norm(D, axis=1)
    D /= dist[:, None]
    return O.astype(np.float32), D.astype(np.float32), emit[e].astype(np.int32), src.astype(np.int32), e, dist


@pytest.mark.parametrize("which", ["cornell", "scene0"])
def test_shadow_occluder_masks_are_conservative(oracle, which):
    """bvh.cpp shadow_occluder_masks: whenever the oracle's closest hit of a
    shadow ray from a point on triangle s towards emitter e is an occluder
    (not the target, no farther than the target point), that occluder's pair
    is in mask[s, e]; the emitter's own
    pair is always in; and the masks do leave pairs out."""
    recs = CORNELL if which == "cornell" else SCENE0
    P = product_scene(recs, device=False)
    Q = oracle.OracleScene(recs)
    tris = P.triangles()
    m = P.shadow_masks()
    O, D, tg, src, e, dist = _shadow_rays(tris, 200000, np.random.RandomState(17))
    t, idx = Q.closest_hit(O, D)
    occ = (idx >= 0) & (idx != tg) & (t <= dist * (1 + 1e-5))  # a hit beyond: the target itself was missed
    assert occ.mean() > 0.001
    bit = np.where(idx >= 0, idx // 2, 0).astype(np.uint32)
    assert np.all((m[src[occ], e[occ]] >> bit[occ]) & 1)
    emit = np.nonzero(tris[:, 56] >= 0)[0]
    for k, et in enumerate(emit):
        assert np.all((m[:, k] >> (et // 2)) & 1)
    assert np.all(m < (1 << ((P.nT + 1) // 2)))
    assert min(bin(int(x)).count("1") for x in m.ravel()) < (P.nT + 1) // 2
