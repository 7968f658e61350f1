"""The N>1 path on CPU: world_size-2 gloo ranks each render their 8-row strips and
bench.gather_frame stitches them on rank 0; the result must equal a single-rank
render bit for bit. The per-rank renderer here is the oracle (no GPU in this test);
on the GPU box the same sharding is checked through the C ABI in
tests/test_gpu_parity.py::test_row_shards_stitch_bit_exactly."""
import os
import socket

import numpy as np
import pytest

W, H, SPP, DEPTH = 40, 36, 2, 8  # H % 8 != 0


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _worker(rank, world, port, q):
    import torch.distributed as dist

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import bench
        from oracle import oracle_py, scene_ref

        prims, (frm, at, vup, fov) = scene_ref.load_json(open(os.path.join(
            os.path.dirname(bench.__file__), "fo-rma_amd", "scenes", "scene_08.min.json")).read())
        cam = oracle_py.camera_look(frm, at, vup, fov, 0.1, W, H)
        mean, _, cnt, _ = oracle_py.render(prims, cam, W, H, SPP, DEPTH, shard_index=rank, shard_count=world)
        frame = bench.gather_frame(mean, rank, world, H)
        total = bench.Barrier(world).sum(cnt["samples"])
        if rank == 0:
            q.put((frame, total))
    finally:
        dist.destroy_process_group()



def test_shard_rows_partition():
    import bench
    for world in (1, 2, 3, 8):
        rows = sorted(sum((bench.shard_rows(1080, r, world) for r in range(world)), []))
        assert rows == list(range(1080))


def test_two_rank_gloo_render_stitches_to_single_rank():
    import torch.multiprocessing as mp
    from oracle import oracle_py, scene_ref

    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    frame, total = q.get(timeout=120)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    prims, (frm, at, vup, fov) = scene_ref.load_json(open(os.path.join(
        os.path.dirname(__file__), "..", "fo-rma_amd", "scenes", "scene_08.min.json")).read())
    cam = oracle_py.camera_look(frm, at, vup, fov, 0.1, W, H)
    full, _, _, _ = oracle_py.render(prims, cam, W, H, SPP, DEPTH)
    assert np.array_equal(frame.view(np.uint32), full.view(np.uint32))
    assert total == W * H * SPP
