"""CPU model of the fast traversal's child-pair steps per query (profiling aid, float64, single
rays): the ordered LBVH as built (Karras splits over the Morton-sorted leaves) against other
binary trees over the same leaf order (which keeps the reference's hit order), on the scene's
primary rays and their shadow rays.  Cube instances are their own boxes, so a ray's closest
hit is the nearest entry among the leaf boxes it hits.
Usage: python tools/tree_quality.py [--scene world8_stress] [--stride 8]"""
import argparse, os, struct, sys
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "gpu-ray-tracer_amd"))
import rtamd


def boxes_of(s):
    inst, im = s.export("instances"), s.export("inst_mesh")
    V, T = s.export("vertices"), s.export("tris")
    info = s.info()
    nm = info["n_meshes"]
    # mesh boxes: vertices referenced by each mesh's triangles (meshes are consecutive triangle runs)
    mesh_of_tri = np.repeat(np.arange(nm), info["n_tris"] // nm)
    mb = []
    for m in range(nm):
        vv = V[T[mesh_of_tri == m, :3].ravel()]
        mb.append((vv.min(0), vv.max(0)))
    lo = np.array([mb[m][0] for m in im]) + inst[:, 4:7]
    hi = np.array([mb[m][1] for m in im]) + inst[:, 4:7]
    return lo.astype(np.float64), hi.astype(np.float64)


def morton_order(lo, hi):
    c = (-(0.5 * (lo + hi))).astype(np.float32)
    b = c.view(np.uint32).astype(np.uint64)
    X, Y, Z = b[:, 0] >> 10, b[:, 1] >> 11, b[:, 2] >> 11
    def spread(v):
        out = np.zeros_like(v)
        for j in range(22):
            out |= ((v >> j) & 1) << (3 * j)
        return out
    key = (spread(X & 0x1fffff) | ((X >> 21) << 63)) | (spread(Z & 0x1fffff) << 1) | (spread(Y & 0x1fffff) << 2)
    return np.argsort(key, kind="stable"), np.sort(key, kind="stable")


def build(keys_or_none, lo, hi, mode):
    """Binary tree over leaf sequence 0..n-1 (already ordered); returns nodes as (lo, hi, a, b)
    children: >= 0 internal node id, < 0 leaf -1-k."""
    n = len(lo)
    nodes = []
    pre_lo = None

    def sah_split(i, j):
        # best split k in (i, j): cost SA(i..k) * (k-i+1) + SA(k+1..j) * (j-k)
        seg_lo, seg_hi = lo[i:j + 1], hi[i:j + 1]
        flo, fhi = np.minimum.accumulate(seg_lo), np.maximum.accumulate(seg_hi)
        blo, bhi = np.minimum.accumulate(seg_lo[::-1])[::-1], np.maximum.accumulate(seg_hi[::-1])[::-1]
        def sa(a, b):
            d = b - a
            return d[:, 0] * d[:, 1] + d[:, 1] * d[:, 2] + d[:, 2] * d[:, 0]
        m = j - i + 1
        left = sa(flo[:-1], fhi[:-1]) * np.arange(1, m)
        right = sa(blo[1:], bhi[1:]) * np.arange(m - 1, 0, -1)
        return i + int(np.argmin(left + right))

    def karras_split(i, j):
        a, b = int(keys_or_none[i]), int(keys_or_none[j])
        if a == b:
            return (i + j) // 2
        hb = (a ^ b).bit_length() - 1
        k = i
        for t in range(i, j):
            if (int(keys_or_none[t + 1]) >> hb) & 1 != (a >> hb) & 1:
                return t
        return (i + j) // 2

    def rec(i, j):
        if i == j:
            return -1 - i
        k = sah_split(i, j) if mode == "sah" else karras_split(i, j) if mode == "karras" else (i + j) // 2
        idx = len(nodes)
        nodes.append(None)
        a, b = rec(i, k), rec(k + 1, j)
        nodes[idx] = (a, b)
        return idx
    rec(0, n - 1)
    # node boxes
    blo = np.zeros((len(nodes), 3)); bhi = np.zeros((len(nodes), 3))
    def box(c):
        return (lo[-1 - c], hi[-1 - c]) if c < 0 else (blo[c], bhi[c])
    for idx in range(len(nodes) - 1, -1, -1):
        (al, ah), (bl, bh) = box(nodes[idx][0]), box(nodes[idx][1])
        blo[idx], bhi[idx] = np.minimum(al, bl), np.maximum(ah, bh)
    return nodes, blo, bhi


def slab(o, d, l, h):
    with np.errstate(divide="ignore", invalid="ignore"):
        inv = 1.0 / d
        t0, t1 = (l - o) * inv, (h - o) * inv
    t0 = np.where(d == 0, -np.inf, t0); t1 = np.where(d == 0, np.inf, t1)
    tn, tf = np.minimum(t0, t1).max(), np.maximum(t0, t1).min()
    return tn <= tf and tf >= 1e-5, max(tn, 0.0)


def trace(tree, lo, hi, o, d, max_t=np.inf, any_hit=False):
    nodes, blo, bhi = tree
    steps, best = 0, np.inf
    stack = [0]
    def box(c):
        return (lo[-1 - c], hi[-1 - c]) if c < 0 else (blo[c], bhi[c])
    while stack:
        nid = stack.pop()
        steps += 1
        kids = []
        for c in nodes[nid]:
            h, t = slab(o, d, *box(c))
            if h and t <= min(best, max_t):
                kids.append((c, t))
        for c, t in kids:                       # DFS order: A then B (B pushed below A)
            pass
        for c, t in reversed(kids):
            if c < 0:
                if t < best and t <= max_t:
                    pass
        # process: leaves now (in order), internals pushed
        push = []
        for c, t in kids:
            if c < 0:
                if t <= min(best, max_t):
                    best = min(best, t)
                    if any_hit:
                        return steps, best
            else:
                push.append(c)
        stack.extend(reversed(push))
    return steps, best


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--scene", default="world8_stress")
    p.add_argument("--stride", type=int, default=8)
    a = p.parse_args()
    s = rtamd.Scene.load_json(os.path.join(ROOT, "scenes", a.scene + ".json"), 1920, 1080)
    lo, hi = boxes_of(s)
    order, keys = morton_order(lo, hi)
    lo, hi = lo[order], hi[order]
    cam = s.export("camera").astype(np.float64)
    pos, near, unit, W, H = cam[0:3], cam[7], cam[8], cam[9], cam[10]
    r, u, f = cam[11:14], cam[14:17], cam[17:20]
    lights = s.export("lights")
    trees = {m: build(keys, lo, hi, m) for m in ("karras", "sah", "median")}
    tot = {m: [0, 0, 0, 0] for m in trees}
    for y in range(0, int(H), a.stride):
        for x in range(0, int(W), a.stride):
            gx, gy = (x + 0.5 - 0.5 * W) / unit, (0.5 * H - y - 0.5) / unit
            d = near * f + gx * r + gy * u
            d /= np.linalg.norm(d)
            for m, tr in trees.items():
                st, t = trace(tr, lo, hi, pos, d)
                tot[m][0] += st; tot[m][1] += 1
                if np.isfinite(t):
                    hp = pos + t * d
                    for L in lights:
                        if L[3] == 0:
                            ld = L[:3] - hp; mt = np.linalg.norm(ld); ld /= mt
                        else:
                            ld = -L[:3] / np.linalg.norm(L[:3]); mt = np.inf
                        st2, _ = trace(tr, lo, hi, hp + 1e-4 * ld, ld, mt, any_hit=True)
                        tot[m][2] += st2; tot[m][3] += 1
    for m, (sp, np_, ss, ns) in tot.items():
        print("%-7s primary steps/ray %.2f  shadow steps/ray %.2f  (rays %d / %d)" % (m, sp / np_, ss / max(1, ns), np_, ns))


if __name__ == "__main__":
    main()
