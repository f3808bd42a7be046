"""Hash (fused launch, z-half waves) vs dense on a small case: where and how the states differ."""
import numpy as np

from tsdf_amd import grid_fusion, hash_fusion, scene


def compare(tag, g, h):
    (Tg, Wg, Cg), (Th, Wh, Ch) = g.get_state(), h.get_state()
    print(tag, "dense", g.stats())
    print(tag, "hash ", h.stats(), h.info())
    z = np.broadcast_to((np.arange(Wg.shape[2]) % 8)[None, None, :], Wg.shape)
    for name, m in (("missing", (Wg > 0) & (Wh == 0)), ("extra", (Wg == 0) & (Wh > 0)),
                    ("diff w", (Wg > 0) & (Wh > 0) & (Wg != Wh)),
                    ("diff t", (Wg == Wh) & (Tg != Th)), ("diff c", (Wg == Wh) & (Cg != Ch))):
        print(tag, name, int(m.sum()), "z<4:", int((m & (z < 4)).sum()), "z>=4:", int((m & (z >= 4)).sum()))
        if m.any():
            for p in np.argwhere(m)[:4]:
                p = tuple(p)
                print("   ", p, "g", Wg[p], Tg[p], Cg[p], "h", Wh[p], Th[p], Ch[p])
            bm = np.unique(np.argwhere(m) // 8, axis=0)
            print("    bricks", len(bm))


def main():
    poses = scene.trajectory(3, seed=0, start=250)
    d, c = scene.render(poses, scene.make_spheres(0), seed=0, start=250)
    d, c = np.ascontiguousarray(d.numpy()), np.ascontiguousarray(c.numpy())
    K = scene.intrinsics()
    bnds = np.array([[0.0, 10.24]] * 3)
    for n in (1, 3):
        g = grid_fusion.TSDFVolume(bnds.copy(), 0.04, defer=False)
        h = hash_fusion.HashTable(bnds.copy(), 0.04, 1 << 18)
        g.integrate_batch(d[:n], c[:n], K, np.linalg.inv(poses[:n]))
        h.integrate_batch(d[:n], c[:n], K, np.linalg.inv(poses[:n]))
        compare(f"batch{n}", g, h)


if __name__ == "__main__":
    main()
