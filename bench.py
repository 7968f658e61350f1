"""Headline benchmark: Msamples/s of the gfx950 path tracer on scenes/scene_08.json at
1920x1080, 256 spp, 8 bounces (BASELINE.json config 3), 1..8 GPUs.

    python bench.py [--gpus N] [--steps K] [--warmup W]
    python -m torch.distributed.run --nnodes=1 --nproc-per-node N --master-addr 127.0.0.1 \
        --master-port P bench.py --gpus N --steps K --warmup W

One process per GPU. A step renders the whole frame: rank r renders the 8-row strips
k with k % N == r (no collective on the data path; each rank's output lands in its own
device buffer). The timed region is K steps bracketed by a barrier and a device
synchronize on both sides; the time is the max over ranks; value = all samples of the
K frames / that time. Inputs (scene, camera) are resident on the device before timing.
Rank 0 prints one JSON line, with the roofline of the trace kernel (HIP-event time on
its own stream) and, at N=1, the oracle CPU baseline timed on a bounded row sample.
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "fo-rma_amd"))

SCENE = "scene_08"
WIDTH, HEIGHT, SPP, DEPTH, SEED = 1920, 1080, 256, 8, 0x5EED
HBM_PEAK_GBS = 8000.0      # MI355X_MICROARCH.md, chip-level parameters (spec)
FP32_PEAK_TFLOPS = 157.3   # MI355X_MICROARCH.md, peak FP32 vector (spec)
PMC_FILE = os.path.join(ROOT, "profiles", "pmc_trace_kernel.json")


def dist_env():
    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local = int(os.environ.get("LOCAL_RANK", str(rank)))
    return rank, world, local


def shard_rows(height, shard, shards, strip=8):
    """Rows of shard `shard`: strips k = shard, shard + shards, ... of `strip` rows."""
    return [y for y in range(height) if (y // strip) % shards == shard]


def gather_frame(mean_rgb, rank, world, height, strip=8):
    """Stitch every rank's strips into rank 0's image (the optional final gather,
    outside the timed region). `mean_rgb` is this rank's full-size [H, W, 3] buffer with
    only its own strips valid. Returns the stitched frame on rank 0, None elsewhere."""
    import numpy as np
    import torch
    import torch.distributed as dist

    if world == 1:
        return mean_rgb
    mine = np.ascontiguousarray(mean_rgb[shard_rows(height, rank, world, strip)])
    parts = [None] * world if rank == 0 else None
    dist.gather_object(mine, parts, dst=0)
    if rank != 0:
        return None
    out = np.empty_like(mean_rgb)
    for r, part in enumerate(parts):
        out[shard_rows(height, r, world, strip)] = part
    return out


def algorithmic_bytes(n_pixels, n_prims):
    """Compulsory HBM bytes of one render, charged to the trace kernel
    that does the work: the scene read once (64 B geometry record + 16 B attenuation +
    16 B material + 4 B scatter class = 100 B per primitive) and each pixel's result
    written once (12 B f32 mean + 3 B u8). The per-sample colour buffer between the
    trace and sum kernels is a design cost, not algorithmic; its bytes show in
    `traffic` (PMC)."""
    return n_prims * 100 + n_pixels * 15


def algorithmic_flops(segments, hits, samples, n_prims):
    """Lower bound of the f32 arithmetic of an all-box scene: per segment
    3 divides (1/d) + 12 per box slab test; per hit 6 (hit point); per sample 24
    (jitter + camera ray)."""
    return segments * (3 + 12 * n_prims) + hits * 6 + samples * 24


class Barrier:
    def __init__(self, world):
        self.world = world
        if world > 1:
            import torch.distributed as dist
            self.dist = dist
            if not dist.is_initialized():
                dist.init_process_group("gloo")

    def __call__(self):
        if self.world > 1:
            self.dist.barrier()

    def max(self, v):
        if self.world == 1:
            return v
        import torch
        t = torch.tensor([float(v)], dtype=torch.float64)
        self.dist.all_reduce(t, op=self.dist.ReduceOp.MAX)
        return float(t.item())

    def sum(self, v):
        if self.world == 1:
            return v
        import torch
        t = torch.tensor([float(v)], dtype=torch.float64)
        self.dist.all_reduce(t, op=self.dist.ReduceOp.SUM)
        return float(t.item())


def device_sync():
    try:
        import torch
        if torch.cuda.is_available():
            torch.cuda.synchronize()
    except Exception:
        pass


def run_gpu_steps(fr, ctx, scene, cam, params, steps, sync_all):
    """Render `steps` frames (this rank's shard); returns per-step stats."""
    stats = []
    for _ in range(steps):
        ctx.render(scene, cam, params)
        stats.append(ctx.sync())
    return stats


def cpu_baseline(budget_s=12.0):
    """The oracle (oracle/oracle.cpp, a C++ restatement of tracer.rs's save_image) on
    this host's cores, over a bounded row sample of the same workload."""
    from oracle import oracle_py, scene_ref
    import forma_rt as fr

    threads = max(1, min(16, len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else os.cpu_count()))
    prims, (frm, at, vup, fov) = scene_ref.load_json(open(fr.scene_path(SCENE)).read())
    cam = oracle_py.camera_look(frm, at, vup, fov, 0.1, WIDTH, HEIGHT)
    # calibrate on two rows per thread (every thread busy), then size the sample to ~budget_s
    step = max(1, HEIGHT // (2 * threads))
    t = time.perf_counter()
    _, _, cnt, rows = oracle_py.render(prims, cam, WIDTH, HEIGHT, SPP, DEPTH, SEED, row_step=step, threads=threads)
    dt = time.perf_counter() - t
    per_row = dt / max(1, rows)  # wall time per row with all threads working
    want_rows = max(threads, int(budget_s / max(per_row, 1e-6)))
    step = max(1, HEIGHT // want_rows)
    t = time.perf_counter()
    _, _, cnt, rows = oracle_py.render(prims, cam, WIDTH, HEIGHT, SPP, DEPTH, SEED, row_step=step, threads=threads)
    dt = time.perf_counter() - t
    return {"value": round(cnt["samples"] / dt / 1e6, 4), "unit": "Msamples/s", "cores": threads, "kind": "port",
            "sample": f"{rows} of {HEIGHT} rows (every {step}th) of {SCENE} {WIDTH}x{HEIGHT} {SPP}spp depth {DEPTH}, "
                      f"{cnt['samples']} samples in {dt:.2f}s, {threads} threads, oracle/oracle.cpp (-O2)",
            "segments_per_sample": round(cnt["segments"] / max(1, cnt["samples"]), 4)}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-budget", type=float, default=12.0)
    ap.add_argument("--verify", action="store_true", help="gather the frame on rank 0 and report a checksum")
    a = ap.parse_args()

    rank, world, local = dist_env()
    # rehearsal only: run every rank on one device (timing is then meaningless)
    if os.environ.get("FR_BENCH_DEVICE") is not None:
        local = int(os.environ["FR_BENCH_DEVICE"])
    if world != a.gpus:
        if world == 1 and a.gpus > 1:
            sys.exit("bench.py --gpus N>1 must be launched with torch.distributed.run (one process per GPU)")
    import forma_rt as fr  # imports torch first, so one HIP runtime serves both

    try:
        import torch
        if torch.cuda.is_available():
            torch.cuda.set_device(local)
    except Exception:
        pass
    barrier = Barrier(world)
    scene = fr.Scene.from_file(fr.scene_path(SCENE), WIDTH, HEIGHT)
    cam = scene.camera
    n_prims = len(scene)
    params = fr.make_params(WIDTH, HEIGHT, SPP, DEPTH, SEED, shard_index=rank, shard_count=world)
    ctx = fr.RenderContext(local)

    run_gpu_steps(fr, ctx, scene, cam, params, a.warmup, device_sync)
    barrier()
    device_sync()
    t0 = time.perf_counter()
    stats = run_gpu_steps(fr, ctx, scene, cam, params, a.steps, device_sync)
    device_sync()
    t1 = time.perf_counter()
    barrier()
    elapsed = barrier.max(t1 - t0)

    my_samples = sum(s["samples"] for s in stats)
    total_samples = barrier.sum(my_samples)
    segs = sum(s["segments"] for s in stats)
    hits = sum(s["hits"] for s in stats)
    kernel_ms = sum(s["kernel_ms"] for s in stats) / max(1, len(stats))
    trace_ms = sum(s["trace_ms"] for s in stats) / max(1, len(stats))  # trace_kernel launches of one frame
    launches = max(1, stats[0]["trace_launches"])                       # sample-block passes
    launch_ms = trace_ms / launches                                       # what rocprof's average reports
    kernel_ms_max = barrier.max(kernel_ms)
    total_segs = barrier.sum(segs)

    # roofline of the dominant kernel (trace_kernel), per launch on this rank
    pixels = len(shard_rows(HEIGHT, rank, world)) * WIDTH
    # a launch renders 1/launches of the frame's samples: its share of the frame's bytes
    bytes_launch = algorithmic_bytes(pixels, n_prims) / launches
    achieved = bytes_launch / (launch_ms * 1e-3) / 1e9
    traffic = None
    if os.path.exists(PMC_FILE):
        try:
            pm = json.load(open(PMC_FILE))
            if pm.get("workload") == f"{SCENE} {WIDTH}x{HEIGHT} {SPP}spp d{DEPTH}" and world == 1:
                traffic = pm.get("hbm_bytes_per_launch")
        except Exception:
            traffic = None
    flops_launch = algorithmic_flops(segs / len(stats), hits / len(stats), my_samples / len(stats), n_prims) / launches
    tflops = flops_launch / (launch_ms * 1e-3) / 1e12

    checksum = None
    if a.verify:
        mean, _ = ctx.download(WIDTH, HEIGHT)
        frame = gather_frame(mean, rank, world, HEIGHT)
        if rank == 0:
            import hashlib
            checksum = hashlib.sha256(frame.tobytes()).hexdigest()[:16]
    if rank != 0:
        return
    value = total_samples / elapsed / 1e6
    out = {
        "metric": "Msamples/sec (pixels×spp) at 1920×1080, 256 spp, 8 bounces; 1/2/4/8 GPU",
        "value": round(value, 3),
        "unit": "Msamples/s",
        "n_gpus": world,
        "steps": a.steps,
        "warmup": a.warmup,
        "ms_per_step": round(elapsed / a.steps * 1e3, 3),
        "higher_is_better": True,
        "scaling": "strong",
        "vs_baseline": None,
        "dtype": "f32",
        "data": "reference scene file scenes/scene_08.json (bundled), fixed RNG seed 0x5EED",
        "config": {"workload": f"{SCENE} {WIDTH}x{HEIGHT} {SPP}spp {DEPTH} bounces (BASELINE config 3)",
                   "scene": SCENE, "width": WIDTH, "height": HEIGHT, "spp": SPP, "max_depth": DEPTH, "seed": SEED,
                   "parallelism": f"row-strips x{world}"},
        "segments_per_sample": round(total_segs / max(1.0, total_samples), 4),
        "kernel_ms": round(kernel_ms, 3),
        "trace_kernel_ms": round(trace_ms, 3),
        "trace_launches": launches,
        "trace_kernel_ms_per_launch": round(launch_ms, 3),
        "kernel_ms_max_rank": round(kernel_ms_max, 3),
        "roofline": {"bound": "hbm", "achieved": round(achieved, 3), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": round(achieved / HBM_PEAK_GBS, 8), "traffic": traffic,
                     "kernel": "trace_kernel", "bytes_per_launch": round(bytes_launch)},
        "valu_roofline": {"bound": "valu", "achieved": round(tflops, 3), "peak": FP32_PEAK_TFLOPS,
                          "unit": "TFLOP/s", "frac": round(tflops / FP32_PEAK_TFLOPS, 5),
                          "flops_per_launch": int(flops_launch), "note": "algorithmic lower bound, DESIGN.md §5"},
    }
    if checksum:
        out["frame_sha256_16"] = checksum
    if world == 1 and not a.no_cpu_baseline:
        out["cpu_baseline"] = cpu_baseline(a.cpu_budget)
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
