"""Worker of tests/test_dist_gpu.py (not a test module): one rank of a world_size-N job that
shares the single GPU of the test box over `gloo` (RCCL needs one GPU per rank), so the
multi-GPU end of the path runs through the real HIP library: a cyclic column shard and a
bucket-range hash shard integrate the same frames, then
  * sharding.mesh_shard  -- border rows exchanged point to point, marching cubes per shard;
  * sharding.gather_meshes / gather_volume -- the union on rank 0;
  * sharding.merge_hash_shards -- live blocks only, imported into one table on rank 0.
Rank 0 saves the results to <out>/dist.npz for the parent test to compare with one unsharded
volume.  With the "cuda" argument every collective buffer is a device tensor (the branches an
RCCL run takes), moved by gloo."""
import contextlib
import io
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)
for p in (os.path.join(REPO, "union-thesis-slam_amd"), os.path.join(REPO, "oracle"), HERE):
    if p not in sys.path:
        sys.path.insert(0, p)

C1 = [[-2.56, 2.56], [-2.56, 2.56], [0.0, 5.12]]


def main(out, buffers="host"):
    import torch.distributed as dist
    from conftest import load_lounge, lounge_intrinsics
    from tsdf_amd import grid_fusion, hash_fusion, sharding
    rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
    dist.init_process_group("gloo")
    # "cuda": the collective buffers in device memory, as under RCCL (sharding.set_buffer_device)
    sharding.set_buffer_device("cuda" if buffers == "cuda" else None)
    K = lounge_intrinsics()
    with contextlib.redirect_stdout(io.StringIO()):
        vol = grid_fusion.TSDFVolume(np.array(C1), 0.04, shard=(rank, world))
        ht = hash_fusion.HashTable(np.array(C1), 0.04, 1 << 16, shard=rank, n_shards=world)
    for f in range(3):
        _, depth, rgb, pose = load_lounge(f)
        vol.integrate(rgb, depth, K, pose)
        ht.integrate(rgb, depth, K, pose)
    # the same frames ingested once on rank 0 and broadcast (sharding.integrate_broadcast)
    with contextlib.redirect_stdout(io.StringIO()):
        vb = grid_fusion.TSDFVolume(np.array(C1), 0.04, shard=(rank, world))
    d = c = T = None
    if rank == 0:
        fr = [load_lounge(f) for f in range(3)]
        d = np.stack([f[0] for f in fr]).astype(np.uint16)
        d[d == 65535] = 0  # the demos' 65.535 m -> 0, as load_lounge's metres have it
        c = np.stack([f[2] for f in fr])
        T = np.linalg.inv(np.stack([f[3] for f in fr]))
    sharding.integrate_broadcast(vb, K, d, c, T, chunk=2)
    same_b = all(np.array_equal(a, b) for a, b in zip(vb.get_state(), vol.get_state()))
    part = sharding.mesh_shard(vol)
    mesh = sharding.gather_meshes(part)
    state = sharding.gather_volume(vol)

    def make_table():
        with contextlib.redirect_stdout(io.StringIO()):
            return hash_fusion.HashTable(np.array(C1), 0.04, 1 << 16)

    merged = sharding.merge_hash_shards(ht, make_table)
    own_blocks = ht.info()["used"]
    tot = sharding.sum_counters({"blocks": int(own_blocks), "bcast_ok": int(same_b)})
    if rank == 0:
        ht_t, ht_w, ht_c = merged.get_state()
        np.savez(os.path.join(out, "dist.npz"), v=mesh[0], f=mesh[1], n=mesh[2], c=mesh[3],
                 t=state[0], w=state[1], col=state[2], ht=ht_t, hw=ht_w, hc=ht_c,
                 merged_used=merged.info()["used"], shard_blocks=tot["blocks"],
                 part_verts=len(part[0]), bcast_ok=tot["bcast_ok"],
                 dev=int(sharding._device().type == "cuda"))
    dist.barrier()
    dist.destroy_process_group()


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2] if len(sys.argv) > 2 else "host")
