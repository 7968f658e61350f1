"""Headline benchmark: Msamples/s of the gfx950 path tracer on scenes/scene_08.json at
1920x1080, 256 spp, 8 bounces (BASELINE.json config 3), 1..8 GPUs.

    python bench.py [--gpus N] [--steps K] [--warmup W]
    python -m torch.distributed.run --nnodes=1 --nproc-per-node N --master-addr 127.0.0.1 \
        --master-port P bench.py --gpus N --steps K --warmup W
    FR_BENCH_DEVICES=0,0 python bench.py --gpus 2     (rehearsal: two shards on device 0)

Two ways to run N > 1 (launch_plan): a plain `python bench.py --gpus N` drives devices
0..N-1 from this one process through fr_mctx, the drop-in's multi-device context
(tracer.rs:83-134's row tiling with a device per band; run_mctx), and reports every
shard's trace time beside the wall time of the whole frames; under torch.distributed.run
each rank is one process per GPU (run_rank). The frames and their stitched image are the
same either way. Per rank: a step renders the rank's strips and gathers them to the host: rank r
renders the 8-row strips k with k % N == r (no collective on the data path) and copies
its strips (f32 means and the u8 image) into page-locked host memory, the "final gather
to host" (BASELINE.md §4). The gather of frame k runs on its own stream while frame k+1
traces; the frames are enqueued back to back with no host wait between them (run_steps;
--sync-each waits for every frame's stats); the timed region ends only when the last
frame's gather has landed. The timed
region is K steps bracketed by a barrier and a device synchronize on both sides; the
time is the max over ranks; value = all samples of the K frames / that time. Inputs
(scene, camera) are resident on the device before timing.

Rank 0 prints one JSON line with:
- frame_span_ms: a frame's trace start to its sum's end (frames overlap when streamed);
- roofline: the trace kernel's binding bound, FP32 VALU: algorithmic FLOP/s (constants
  frozen in fo-rma_amd/csrc/flops.h, times the kernel's exact counters) against the
  157.3 TFLOP/s peak, plus the VALU issue fraction and HBM traffic read from rocprofv3
  hardware counters in this run (a child process, N=1 only);
- hbm_roofline: algorithmic bytes per launch against 8 TB/s (the north star's ask);
- cpu_baseline (N=1): the oracle on this host's cores, all of them and one; its `c1`
  entry is BASELINE config C1 (scene_01 256x256/4 spp/4 bounces, the reference's CPU
  case) in full on the oracle (1 thread, all threads) and on the GPU, compared bit for bit.
"""
import argparse
import glob
import json
import math
import os
import re
import shutil
import signal
import subprocess
import sys
import tempfile
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "fo-rma_amd"))

SCENE = "scene_08"
WIDTH, HEIGHT, SPP, DEPTH, SEED = 1920, 1080, 256, 8, 0x5EED
HBM_PEAK_GBS = 8000.0      # MI355X_MICROARCH.md, chip-level parameters (spec)
FP32_PEAK_TFLOPS = 157.3   # MI355X_MICROARCH.md, peak FP32 vector (spec)
# The ceiling parity allows: no FMA contraction, so one f32 op per lane per issue slot:
# 256 CUs x 4 SIMDs x 32 lanes/clk (a wave64 VALU instruction issues over 2 cycles,
# MI355X_MICROARCH.md) x 2.4 GHz = 78.6 Tops/s, half the 157.3 TFLOP/s FMA peak. (SURVEY.md
# §8d's 39.3 assumed 157.3 counted packed FMA, i.e. 16 lanes/clk per SIMD.)
NO_FMA_PEAK_TOPS = 78.6
N_SIMDS = 1024             # 256 CUs x 4 SIMDs; a wave64 VALU instruction issues over 2 cycles
FLOPS_H = os.path.join(ROOT, "fo-rma_amd", "csrc", "flops.h")


def dist_env(env=None):
    env = os.environ if env is None else env
    rank = int(env.get("RANK", "0"))
    world = int(env.get("WORLD_SIZE", "1"))
    local = int(env.get("LOCAL_RANK", str(rank)))
    return rank, world, local


def launch_plan(gpus, env=None):
    """How this process runs `gpus` GPUs. Returns {"mode", "rank", "world", "devices"}:
    - "ranks": launched by torch.distributed.run (WORLD_SIZE > 1), one process per GPU;
      this rank renders shard RANK of WORLD_SIZE on device LOCAL_RANK (FR_BENCH_DEVICE
      overrides it: every rank on one device, a rehearsal);
    - "mctx": a plain `python bench.py --gpus N` (N > 1): this one process drives fr_mctx
      over devices 0..N-1, shard i on device i — the drop-in's own multi-device path
      (tracer.rs:83-134's row tiling, one device per band); FR_BENCH_DEVICES=0,0,...
      (N entries) lists the devices instead, so one GPU rehearses an N-shard run;
    - "single": N = 1 (FR_BENCH_DEVICES=d picks the device).
    Raises SystemExit on an inconsistent request."""
    env = os.environ if env is None else env
    rank, world, local = dist_env(env)
    if gpus < 1:
        raise SystemExit(f"bench.py: --gpus must be >= 1, got {gpus}")
    if world > 1:
        if gpus != world:
            raise SystemExit(f"bench.py: --gpus {gpus} under a launcher with WORLD_SIZE={world}")
        dev = int(env["FR_BENCH_DEVICE"]) if env.get("FR_BENCH_DEVICE") not in (None, "") else local
        return {"mode": "ranks", "rank": rank, "world": world, "devices": [dev]}
    spec = env.get("FR_BENCH_DEVICES", "")
    if spec.strip():
        devices = [int(x) for x in spec.split(",") if x.strip()]
        if len(devices) != gpus or min(devices) < 0:
            raise SystemExit(f"bench.py: FR_BENCH_DEVICES={spec!r} must list {gpus} device ids")
    else:
        dev = int(env["FR_BENCH_DEVICE"]) if gpus == 1 and env.get("FR_BENCH_DEVICE") not in (None, "") else 0
        devices = [dev] if gpus == 1 else list(range(gpus))
    return {"mode": "mctx" if gpus > 1 else "single", "rank": 0, "world": 1, "devices": devices}


def shard_rows(height, shard, shards, strip=8):
    """Rows of shard `shard`: strips k = shard, shard + shards, ... of `strip` rows."""
    return [y for y in range(height) if (y // strip) % shards == shard]


def gather_frame(mean_rgb, rank, world, height, strip=8):
    """Stitch every rank's strips into rank 0's image (after timing).
    `mean_rgb` is this rank's full-size [H, W, 3] buffer with only its own strips valid.
    Returns the stitched frame on rank 0, None elsewhere."""
    import numpy as np
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


# ---- algorithmic work model ----------------------------------------------------

def flop_constants(path=FLOPS_H):
    """The `constexpr double kFlop...` / `k...Tries` constants of flops.h, evaluated in
    order (later ones may use earlier ones)."""
    consts = {}
    for name, expr in re.findall(r"constexpr double (k\w+) = ([^;]+);", open(path).read()):
        consts[name] = float(eval(expr, {"__builtins__": {}}, dict(consts)))
    return consts


def algorithmic_flops(c, counts, prim_kinds, pixels, scatter="Lambert"):
    """f32 operations of one render of an in-order-loop scene (flops.h's formula).
    counts: segments / hits / scatters / samples; prim_kinds: kind name -> count. The
    winner-kind and scatter-class terms use the scene's single kind and class (scene_08:
    boxes, lambertian)."""
    seg = c["kFlopSegment"] + (c["kFlopSegmentSphere"] if prim_kinds.get("Sphere") else 0.0)
    seg += c.get("kFlopSegmentBox", 0.0) if prim_kinds.get("Box") else 0.0
    seg += sum(n * c[f"kFlopTest{k}"] for k, n in prim_kinds.items())
    (kind,) = [k for k, n in prim_kinds.items() if n]
    return (counts["segments"] * seg + counts["hits"] * c[f"kFlopHit{kind}"]
            + counts["scatters"] * (c[f"kFlopScatter{scatter}"] + c["kFlopUnwind"])
            + (counts["segments"] - counts["hits"]) * c["kFlopSky"]
            + counts["samples"] * (c["kFlopCamera"] + c["kFlopSum"]) + pixels * c["kFlopPixel"])


def algorithmic_bytes(n_pixels, n_prims):
    """Compulsory HBM bytes of one render: the scene read once (64 B
    geometry record + 16 B attenuation + 16 B material + 4 B scatter class = 100 B per
    primitive) and each pixel's result written once (12 B f32 mean + 3 B u8)."""
    return n_prims * 100 + n_pixels * 15


# ---- in-run hardware counters (rocprofv3, child process) ----------------------

PMC_PASSES = (
    ("sq", ["SQ_INSTS_VALU", "SQ_WAVES", "SQ_INSTS_SALU", "SQ_INSTS_LDS", "SQ_BUSY_CYCLES", "GRBM_GUI_ACTIVE"]),
    ("fetch", ["FETCH_SIZE"]),
    ("write", ["WRITE_SIZE"]),
)


def _run_killable(cmd, timeout, env, log):
    with open(log, "w") as f:
        p = subprocess.Popen(cmd, stdout=f, stderr=subprocess.STDOUT, env=env, start_new_session=True)
        try:
            return p.wait(timeout=timeout)
        except subprocess.TimeoutExpired:
            os.killpg(p.pid, signal.SIGKILL)
            p.wait()
            return -9


def pmc_in_run(frames=2, timeout=150, scene_jit=False):
    """Per-launch counters of trace_kernel for this workload: one rocprofv3 pass per
    counter group (never combined with other traces), each with --kernel-trace --stats
    for that pass's own launch durations. Returns a dict, or {"error": ...}."""
    exe = shutil.which("rocprofv3")
    if not exe:
        return {"error": "rocprofv3 not found"}
    out = tempfile.mkdtemp(prefix="fr_pmc_")
    env = dict(os.environ, FR_NO_TORCH="1", TMPDIR="/tmp")
    if scene_jit:
        env["FR_SCENE_JIT"] = "1"  # the profiled frames run the same (scene-specialised) kernel
    prog = [sys.executable, os.path.join(ROOT, "tools", "pmc_frame.py"), SCENE, str(WIDTH), str(HEIGHT), str(SPP),
            str(DEPTH), str(frames)]
    res = {}
    for tag, counters in PMC_PASSES:
        d = os.path.join(out, tag)
        rc = _run_killable([exe, "--pmc", *counters, "--kernel-trace", "--stats", "-d", d, "-o", tag,
                            "--output-format", "csv", "--", *prog], timeout, env, d + ".log")
        if rc != 0:
            return {"error": f"rocprofv3 pass {tag} exited {rc}", "log": open(d + ".log").read()[-800:]}
        vals = {}
        for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
            import csv
            for r in csv.DictReader(open(f)):
                if "trace_kernel" in r["Kernel_Name"]:
                    vals.setdefault(r["Counter_Name"], []).append(float(r["Counter_Value"]))
        for f in glob.glob(os.path.join(d, "**", "*kernel_stats.csv"), recursive=True):
            import csv
            for r in csv.DictReader(open(f)):
                if "trace_kernel" in r["Name"]:
                    res[f"{tag}_avg_ns"] = float(r["AverageNs"])
        for k, v in vals.items():
            res[k] = sum(v) / len(v)
    keep = os.environ.get("FR_BENCH_PMC_DIR")
    if keep:
        shutil.copytree(out, keep, dirs_exist_ok=True)
    shutil.rmtree(out, ignore_errors=True)
    return res


def valu_issue(pmc):
    """SQ_INSTS_VALU (wave instructions per launch) against the chip's issue rate over the
    profiled launch: 1024 SIMDs x clock / 2 cycles, the clock from GRBM_GUI_ACTIVE (summed
    over the 8 XCDs) over the same launch's duration."""
    ns = pmc.get("sq_avg_ns")
    if not ns or "SQ_INSTS_VALU" not in pmc or "GRBM_GUI_ACTIVE" not in pmc:
        return None
    clk = pmc["GRBM_GUI_ACTIVE"] / 8 / (ns * 1e-9)
    peak = N_SIMDS * clk / 2
    return {"insts_per_launch": pmc["SQ_INSTS_VALU"], "launch_ns": ns, "clock_ghz": round(clk / 1e9, 3),
            "frac": round(pmc["SQ_INSTS_VALU"] / (ns * 1e-9) / peak, 4),
            "source": "rocprofv3 --pmc SQ_INSTS_VALU GRBM_GUI_ACTIVE --kernel-trace in this run"}


def hbm_traffic(pmc):
    """HBM bytes per trace launch: 2 x FETCH_SIZE (gfx950 tallies a 128-B read at 64 B,
    MI355X_MICROARCH.md §HBM) + WRITE_SIZE, both in KB, separate passes."""
    if "FETCH_SIZE" not in pmc or "WRITE_SIZE" not in pmc:
        return None
    return (2 * pmc["FETCH_SIZE"] + pmc["WRITE_SIZE"]) * 1024


# ---- CPU baseline ----------------------------------------------------------------

def host_info():
    info = {"nproc": os.cpu_count(),
            "affinity": len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else os.cpu_count()}
    try:
        q, per = open("/sys/fs/cgroup/cpu.max").read().split()
        info["cgroup_cpus"] = None if q == "max" else round(int(q) / int(per), 2)
    except Exception:
        info["cgroup_cpus"] = None
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                info["model"] = line.split(":", 1)[1].strip()
                break
    except Exception:
        pass
    return info


def cpu_threads(host):
    """Threads the CPU baseline runs on: the affinity mask capped at the cgroup CPU quota
    (rounded up), i.e. the cores this process can actually use at once."""
    n = max(1, host["affinity"])
    q = host.get("cgroup_cpus")
    if q:
        n = min(n, max(1, math.ceil(q)))
    return n


def cpu_baseline(budget_s=12.0, single_s=3.0):
    """The oracle (oracle/oracle.cpp, a C++ restatement of tracer.rs's save_image) on
    this host, over a bounded row sample of the same workload: `cpu-omp` (rows and
    32-pixel chunks over threads, the render_mt shape) on as many threads as the process
    has CPUs (affinity mask capped at the cgroup quota: `cores`), the same sample on every
    thread of the affinity mask when that is more (`oversubscribed`, reported only), and
    `cpu-ref` on one thread (the save_image shape) for at least 2 s."""
    from oracle import oracle_py, scene_ref
    import forma_rt as fr

    host = host_info()
    threads = cpu_threads(host)
    prims, (frm, at, vup, fov) = scene_ref.load_json(open(fr.scene_path(SCENE)).read())
    cam = oracle_py.camera_look(frm, at, vup, fov, 0.1, WIDTH, HEIGHT)

    def timed(step, nthreads, col_step=1):
        t = time.perf_counter()
        _, _, cnt, rows = oracle_py.render(prims, cam, WIDTH, HEIGHT, SPP, DEPTH, SEED, row_step=step,
                                           threads=nthreads, col_step=col_step)
        return cnt, rows, time.perf_counter() - t

    # calibrate on 8 spread rows, about two 32-pixel chunks per thread, then size the
    # sample to the budget
    cnt, rows, dt = timed(HEIGHT // 8, threads, col_step=max(1, 8 * WIDTH // (64 * threads)))
    per_sample = dt / max(1, cnt["samples"])
    want_rows = max(1, int(budget_s / per_sample / (WIDTH * SPP)))
    step = max(1, HEIGHT // want_rows)
    cnt, rows, dt = timed(step, threads)
    if dt < 0.5 * budget_s and step > 1:  # the calibration overstated the cost: widen once
        step = max(1, int(step * dt / budget_s))
        cnt, rows, dt = timed(step, threads)
    omp = {"value": round(cnt["samples"] / dt / 1e6, 4), "unit": "Msamples/s", "cores": threads, "kind": "port",
           "sample": f"{rows} of {HEIGHT} rows (every {step}th) of {SCENE} {WIDTH}x{HEIGHT} {SPP}spp depth {DEPTH}, "
                     f"{cnt['samples']} samples in {dt:.2f}s on {threads} threads, oracle/oracle.cpp (-O2)",
           "threads_rule": "min(affinity mask, ceil(cgroup CPU quota))",
           "segments_per_sample": round(cnt["segments"] / max(1, cnt["samples"]), 4), "host": host}
    if host["affinity"] > threads:
        cnt2, rows2, dt2 = timed(step, host["affinity"])
        omp["oversubscribed"] = {"value": round(cnt2["samples"] / dt2 / 1e6, 4), "unit": "Msamples/s",
                                 "threads": host["affinity"],
                                 "sample": f"the same {rows2} rows on every thread of the affinity mask "
                                           f"({host['affinity']} threads in a {host.get('cgroup_cpus')}-CPU quota): "
                                           f"{cnt2['samples']} samples in {dt2:.2f}s"}
    # one thread: the same rows, every cstep-th pixel, sized to `single_s` seconds from the
    # multi-thread rate (a thread does at most that rate / 1 and at least / threads)
    per_sample_1 = dt / max(1, cnt["samples"]) * threads
    pix = rows * WIDTH
    cstep = max(1, int(pix * SPP * per_sample_1 / single_s))
    cnt1, rows1, dt1 = timed(step, 1, col_step=cstep)
    while dt1 < 2.0 and cstep > 1:  # scaling was sub-linear: a larger sample, until >= 2 s
        cstep = max(1, int(cstep * dt1 / single_s))
        cnt1, rows1, dt1 = timed(step, 1, col_step=cstep)
    omp["single_thread"] = {"value": round(cnt1["samples"] / dt1 / 1e6, 4), "unit": "Msamples/s", "cores": 1,
                            "kind": "port", "sample": f"the same {rows1} rows, every {cstep}th pixel: "
                                                      f"{cnt1['samples']} samples in {dt1:.2f}s "
                                                      "(cpu-ref, the save_image shape)"}
    return omp


def config_c1(ctx, steps=5):
    """BASELINE config C1 (scene_01 at 256x256, 4 spp, 4 bounces; the reference's CPU
    plumbing case, tracer.rs:160-187) in full: the oracle as `cpu-ref` (1 thread) and
    `cpu-omp` (every core of the affinity mask), and the HIP path on this rank's device
    (render + gather per step, after one warm-up), with the frames compared bit for bit."""
    import numpy as np

    from oracle import oracle_py, scene_ref
    import forma_rt as fr

    w, h, spp, depth, name = 256, 256, 4, 4, "scene_01"
    prims, (frm, at, vup, fov) = scene_ref.load_json(open(fr.scene_path(name)).read())
    cam = oracle_py.camera_look(frm, at, vup, fov, 0.1, w, h)
    threads = cpu_threads(host_info())
    out = {"config": f"{name} {w}x{h} {spp}spp {depth} bounces (BASELINE config 1), full frame", "samples": w * h * spp}
    ref = None
    for label, nt in (("cpu_ref", 1), ("cpu_omp", threads)):
        t = time.perf_counter()
        omean, ou8, cnt, _ = oracle_py.render(prims, cam, w, h, spp, depth, SEED, threads=nt)
        dt = time.perf_counter() - t
        ref = ref or (omean, ou8)
        out[label] = {"value": round(cnt["samples"] / dt / 1e6, 4), "unit": "Msamples/s", "cores": nt,
                      "kind": "port", "ms": round(dt * 1e3, 3)}
    sc = fr.Scene.from_file(fr.scene_path(name), w, h)
    params = fr.make_params(w, h, spp, depth, SEED)
    frame = fr.PinnedFrame(w, h)
    run_steps(ctx, sc, sc.camera, params, frame, 1)
    device_sync(ctx)
    t = time.perf_counter()
    run_steps(ctx, sc, sc.camera, params, frame, steps)
    device_sync(ctx)
    dt = (time.perf_counter() - t) / steps
    out["gpu"] = {"value": round(w * h * spp / dt / 1e6, 3), "unit": "Msamples/s", "ms_per_step": round(dt * 1e3, 4),
                  "step": "render + D2H gather"}
    mean, u8 = frame.mean.reshape(h, w, 3), frame.u8.reshape(h, w, 3)
    out["gpu"]["max_abs_diff_vs_cpu_ref"] = float(np.max(np.abs(mean - ref[0])))
    out["gpu"]["u8_identical"] = bool(np.array_equal(u8, ref[1]))
    frame.close()
    return out


# ---- the run --------------------------------------------------------------------

class Barrier:
    def __init__(self, world):
        self.world = world
        if world > 1:
            import torch.distributed as dist
            self.dist = dist
            if not dist.is_initialized():
                # gloo's connection message goes to fd 1: keep stdout for the one JSON line
                sys.stdout.flush()
                saved = os.dup(1)
                os.dup2(2, 1)
                try:
                    dist.init_process_group("gloo")
                finally:
                    os.dup2(saved, 1)
                    os.close(saved)

    def __call__(self):
        if self.world > 1:
            self.dist.barrier()

    def reduce(self, v, op):
        if self.world == 1:
            return v
        import torch
        t = torch.tensor([float(v)], dtype=torch.float64)
        self.dist.all_reduce(t, op=op)
        return float(t.item())

    def max(self, v):
        return v if self.world == 1 else self.reduce(v, self.dist.ReduceOp.MAX)

    def sum(self, v):
        return v if self.world == 1 else self.reduce(v, self.dist.ReduceOp.SUM)


def device_sync(ctx):
    """Every stream of the render context, then the whole device."""
    import torch
    ctx.wait()
    if torch.cuda.is_available():
        torch.cuda.synchronize()


def run_steps(ctx, scene, cam, params, frame, steps, sync_each=False):
    """Render `steps` frames of this rank's shard, each followed by its asynchronous gather
    into the pinned host frame; returns per-step stats.

    By default the frames are enqueued back to back with no host wait between them, as a
    renderer streaming frames runs: the context's streams order frame k+1's trace after
    frame k's sum, its sum after frame k's gather (fr_ctx_download_async), so every frame
    is rendered and gathered in full, and the GPU does not idle while the host reads a
    frame's counters and enqueues the next. The counters and event times are then the last
    frame's, which are every frame's (the same deterministic work). sync_each=True waits
    for each frame's stats before enqueueing the next (round-2 behaviour, --sync-each)."""
    if sync_each:
        stats = []
        for _ in range(steps):
            ctx.render(scene, cam, params)
            stats.append(ctx.sync())
            ctx.download_async(frame)
        return stats
    for _ in range(steps):
        ctx.render(scene, cam, params)
        ctx.download_async(frame)
    return [ctx.sync()] * steps if steps else []



def scene_kinds(fr, scene):
    """Primitive count per kind name (flops.h's kFlopTest<Kind> names)."""
    kinds = {}
    for p in scene.prims():
        name = {fr.FR_SPHERE: "Sphere", fr.FR_PLANE: "Plane", fr.FR_AABB: "Box", fr.FR_OBB: "Obb",
                fr.FR_TRIANGLE: "Triangle"}.get(p.kind)
        if name:
            kinds[name] = kinds.get(name, 0) + 1
    return kinds


def rooflines(counts, kinds, pixels, n_prims, launches, launch_ms, traffic=None, issue=None):
    """The trace kernel's rooflines per launch on one device: FP32 VALU (the binding bound)
    and HBM (the north star's ask), from the algorithmic work of `counts` over `launches`
    launches of `launch_ms` each."""
    c = flop_constants()
    flops_launch = algorithmic_flops(c, counts, kinds, pixels) / launches
    tflops = flops_launch / (launch_ms * 1e-3) / 1e12
    bytes_launch = algorithmic_bytes(pixels, n_prims) / launches
    gbs = bytes_launch / (launch_ms * 1e-3) / 1e9
    roof = {"bound": "valu", "achieved": round(tflops, 3), "peak": FP32_PEAK_TFLOPS, "unit": "TFLOP/s",
            "frac": round(tflops / FP32_PEAK_TFLOPS, 5), "traffic": round(traffic) if traffic else None,
            "peak_no_fma": NO_FMA_PEAK_TOPS, "frac_no_fma": round(tflops / NO_FMA_PEAK_TOPS, 5),
            "peak_no_fma_rule": "1024 SIMDs x 32 lanes/clk x 2.4 GHz (no contraction: 1 op per lane-slot)",
            "kernel": "trace_kernel", "flops_per_launch": round(flops_launch),
            "flop_model": "fo-rma_amd/csrc/flops.h x exact counters", "valu_issue": issue}
    hbm = {"bound": "hbm", "achieved": round(gbs, 3), "peak": HBM_PEAK_GBS, "unit": "GB/s",
           "frac": round(gbs / HBM_PEAK_GBS, 8), "bytes_per_launch": round(bytes_launch),
           "traffic": round(traffic) if traffic else None,
           "measured_gbs": round(traffic / (launch_ms * 1e-3) / 1e9, 2) if traffic else None}
    return roof, hbm


def base_line(a, n_gpus, value, elapsed, parallelism):
    return {
        "metric": "Msamples/sec (pixels×spp) at 1920×1080, 256 spp, 8 bounces; 1/2/4/8 GPU",
        "value": round(value, 3),
        "unit": "Msamples/s",
        "n_gpus": n_gpus,
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
                   "parallelism": parallelism},
    }


def frame_hash(mean):
    import hashlib
    return hashlib.sha256(mean.tobytes()).hexdigest()[:16]


def compare_with_n1(stitched, n1):
    """The N > 1 line's self-check: the frame stitched from the N shards against the same
    frame rendered whole on one device (the RNG is keyed by global pixel, so the strips of
    tracer.rs:83-134's row tiling must give the N = 1 image bit for bit)."""
    a, b = frame_hash(stitched), frame_hash(n1)
    return {"frame_sha256_16": a, "n1_frame_sha256_16": b, "frame_matches_n1": a == b}


def render_n1_frame(fr, device, scene, cam, no_scene_jit):
    """The whole frame on one context of `device` (after the timed region): the N = 1
    reference for compare_with_n1."""
    ctx = fr.RenderContext(device)
    try:
        ctx.render(scene, cam, fr.make_params(WIDTH, HEIGHT, SPP, DEPTH, SEED, scene_jit=not no_scene_jit))
        ctx.sync()
        mean, _ = ctx.download(WIDTH, HEIGHT)
    finally:
        ctx.close()
    return mean


def run_mctx(a, plan, torch, fr):
    """N > 1 in one process: fr_mctx over plan["devices"], shard i of N on entry i, every
    frame's strips gathered asynchronously into the context's page-locked host frame.
    A step = one whole frame on all devices (enqueued back to back, no host wait between
    frames); the timed region ends when every device's last gather has landed, so the wall
    time is the slowest shard's. Per-shard HIP-event times of every trace launch and
    render of the K frames are reported beside it."""
    devices = plan["devices"]
    n = len(devices)
    have = fr.device_count()
    if have < max(devices) + 1:
        raise SystemExit(f"bench.py --gpus {n}: devices {devices} requested, {have} present "
                         f"(FR_BENCH_DEVICES=0,0,... rehearses an {n}-shard run on one device)")
    rehearsal = len(set(devices)) < n

    rendered = [False]

    def sync_all():
        if rendered[0]:
            mc.sync()
        if torch.cuda.is_available():
            for d in sorted(set(devices)):
                torch.cuda.synchronize(d)

    scene = fr.Scene.from_file(fr.scene_path(SCENE), WIDTH, HEIGHT)
    cam = scene.camera
    kinds = scene_kinds(fr, scene)
    mc = fr.MultiContext(devices)
    params = fr.make_params(WIDTH, HEIGHT, SPP, DEPTH, SEED, scene_jit=not a.no_scene_jit)
    ctxs = [mc.context(i) for i in range(n)]
    tp = time.perf_counter()
    jits = [c.prepare(scene, cam, fr.make_params(WIDTH, HEIGHT, SPP, DEPTH, SEED, shard_index=i, shard_count=n,
                                                 scene_jit=not a.no_scene_jit)) for i, c in enumerate(ctxs)]
    prepare_ms = (time.perf_counter() - tp) * 1e3
    for _ in range(a.warmup):
        mc.render(scene, cam, params)
        rendered[0] = True
        if a.sync_each:
            mc.sync()
    if a.warmup:
        sync_all()
    for c in ctxs:
        c.trace_log(True)
    sync_all()
    t0 = time.perf_counter()
    host_ms = 0.0  # host time inside fr_mctx_render (enqueueing every shard and gather)
    for _ in range(a.steps):
        th = time.perf_counter()
        mc.render(scene, cam, params)
        host_ms += (time.perf_counter() - th) * 1e3
        rendered[0] = True
        if a.sync_each:
            mc.sync()
    sync_all()  # every shard's last gather has landed
    elapsed = time.perf_counter() - t0
    total = mc.sync()
    shards = []
    for i, c in enumerate(ctxs):
        st = c.sync()
        launches_ms = c.trace_log_read()
        frames_ms = c.trace_log_read(frames=True)
        c.trace_log(False)
        shards.append({"shard": i, "device": devices[i], "samples": st["samples"], "segments": st["segments"],
                       "hits": st["hits"], "scatters": st["scatters"],
                       "segments_per_sample": round(st["segments"] / max(1, st["samples"]), 4),
                       "trace_launches": st["trace_launches"],
                       "occupancy": st["occupancy"],
                       "trace_ms_per_launch": round(sum(launches_ms) / max(1, len(launches_ms)), 4),
                       "trace_ms_min_max": [round(min(launches_ms), 4), round(max(launches_ms), 4)]
                       if launches_ms else None,
                       "frame_span_ms": round(sum(frames_ms) / max(1, len(frames_ms)), 4),
                       "launches_logged": len(launches_ms)})
    mean, _ = mc.frame()
    value = total["samples"] * a.steps / elapsed / 1e6
    slow = max(shards, key=lambda s: s["trace_ms_per_launch"] * s["trace_launches"])
    launches = max(1, slow["trace_launches"])
    # a shard's consecutive traces may overlap (frame pipeline): cap at the step time
    launch_ms = min(slow["trace_ms_per_launch"], elapsed / max(1, a.steps) * 1e3)
    pixels = len(shard_rows(HEIGHT, slow["shard"], n)) * WIDTH
    roof, hbm = rooflines({k: slow[k] for k in ("segments", "hits", "scatters", "samples")}, kinds, pixels,
                          len(scene), launches, launch_ms)
    roof["shard"] = slow["shard"]
    out = base_line(a, n, value, elapsed, f"row-strips x{n}, one process, fr_mctx over devices {devices}"
                    + (" (REHEARSAL: devices repeat)" if rehearsal else ""))
    out.update({
        "launch": "one process (fr_mctx), no launcher" + (" — REHEARSAL: devices repeat, timing is not an "
                                                           "N-GPU measurement" if rehearsal else ""),
        "rehearsal": rehearsal,
        "step": "one frame: every shard's render + D2H gather of its f32 means and u8 image into one page-locked "
                "host frame",
        "host_sync": "each step" if a.sync_each else "after the K steps (frames streamed back to back)",
        "segments_per_sample": round(total["segments"] / max(1, total["samples"]), 4),
        "scatters_per_sample": round(total["scatters"] / max(1, total["samples"]), 4),
        "host_enqueue_ms_per_frame": round(host_ms / max(1, a.steps), 4),
        "trace_kernel_ms_per_launch_max_shard": slow["trace_ms_per_launch"],
        "trace_kernel_ms_per_launch_min_shard": min(s["trace_ms_per_launch"] for s in shards),
        "shards": shards,
        "timing_source": "wall clock over the K frames (all devices synchronised on both sides); per-shard HIP "
                         "events around every trace launch and render (fr_ctx_trace_log)",
        "scene_kernel": {"specialised": all(j["used"] for j in jits),
                         "hiprtc_compiled": sum(1 for j in jits if j["compiled"]),
                         "get_ms": [round(j["ms"], 1) for j in jits], "prepare_ms": round(prepare_ms, 1)},
        "roofline": roof,
        "hbm_roofline": hbm,
    })
    mc.close()
    out.update(compare_with_n1(mean, render_n1_frame(fr, devices[0], scene, cam, a.no_scene_jit)))
    return out


def run_rank(a, plan, torch, fr):
    """N = 1, or one rank of a torch.distributed.run launch (one process per GPU)."""
    rank, world, local = plan["rank"], plan["world"], plan["devices"][0]
    if torch.cuda.is_available():
        torch.cuda.set_device(local)
    barrier = Barrier(world)
    scene = fr.Scene.from_file(fr.scene_path(SCENE), WIDTH, HEIGHT)
    cam = scene.camera
    n_prims = len(scene)
    kinds = scene_kinds(fr, scene)
    params = fr.make_params(WIDTH, HEIGHT, SPP, DEPTH, SEED, shard_index=rank, shard_count=world,
                            scene_jit=not a.no_scene_jit)
    ctx = fr.RenderContext(local)
    frame = fr.PinnedFrame(WIDTH, HEIGHT)
    # Set-up before any frame, untimed like the scene upload: the scene's device copy, the
    # buffers and (FR_FLAG_SCENE_JIT) the trace kernel specialised to this scene's records —
    # hiprtc compile or the on-disk code-object cache (fo-rma_amd/csrc/jit.cpp).
    tp = time.perf_counter()
    jit = ctx.prepare(scene, cam, params)
    prepare_ms = (time.perf_counter() - tp) * 1e3

    run_steps(ctx, scene, cam, params, frame, a.warmup, a.sync_each)
    device_sync(ctx)
    ctx.trace_log(True)  # HIP events around every trace launch and render of the K frames
    barrier()
    device_sync(ctx)
    t0 = time.perf_counter()
    stats = run_steps(ctx, scene, cam, params, frame, a.steps, a.sync_each)
    device_sync(ctx)  # the last frame's gather has landed
    t1 = time.perf_counter()
    barrier()
    elapsed = barrier.max(t1 - t0)
    launch_log = ctx.trace_log_read()             # every trace launch of the K frames (ms)
    frame_log = ctx.trace_log_read(frames=True)   # every render of the K frames (ms)
    ctx.trace_log(False)

    n = max(1, len(stats))
    my_samples = sum(s["samples"] for s in stats)
    total_samples = barrier.sum(my_samples)
    counts = {k: sum(s[k] for s in stats) / n for k in ("segments", "hits", "scatters", "samples")}
    launches = max(1, stats[0]["trace_launches"])              # sample-block passes
    # means over all K frames from the launch log (not the last frame's events)
    kernel_ms = sum(frame_log) / max(1, len(frame_log))        # the render on its streams (trace + sum)
    launch_ms = sum(launch_log) / max(1, len(launch_log))      # what rocprof's average reports
    # A small shard's consecutive traces overlap (the frame pipeline): a
    # launch's own events then span part of its neighbour, so the roofline's kernel time is
    # capped at the step time (conservative).
    launch_ms_events = launch_ms
    launch_ms = min(launch_ms, elapsed / max(1, a.steps) * 1e3)
    trace_ms = launch_ms * launches                            # trace_kernel launches of one frame
    kernel_ms_max = barrier.max(kernel_ms)
    total_segs = barrier.sum(counts["segments"] * n)
    pixels = len(shard_rows(HEIGHT, rank, world)) * WIDTH

    # every run reports its frame's hash; N > 1 stitches the shards on rank 0 (after the timed
    # region) and checks them against the whole frame rendered on rank 0's device
    frame_img = gather_frame(frame.mean, rank, world, HEIGHT)
    check = None
    if rank == 0:
        check = ({"frame_sha256_16": frame_hash(frame_img)} if world == 1 else
                 compare_with_n1(frame_img, render_n1_frame(fr, local, scene, cam, a.no_scene_jit)))
    if rank != 0:
        return None
    pmc = pmc_in_run(scene_jit=jit["used"]) if (world == 1 and not a.no_pmc) else {}
    issue = valu_issue(pmc)
    traffic = hbm_traffic(pmc)
    value = total_samples / elapsed / 1e6
    roof, hbm = rooflines(counts, kinds, pixels, n_prims, launches, launch_ms, traffic, issue)
    # FR_BENCH_DEVICE under the launcher puts every rank on one device (launch_plan): a
    # rehearsal of the N-rank path, not an N-GPU measurement
    rehearsal = world > 1 and os.environ.get("FR_BENCH_DEVICE") not in (None, "")
    out = base_line(a, world, value, elapsed, f"row-strips x{world}"
                    + (" (REHEARSAL: every rank on one device)" if rehearsal else ""))
    out.update({
        "launch": "single process" if world == 1 else f"torch.distributed.run, {world} ranks (one process per GPU)",
        "rehearsal": rehearsal,
        "step": "render of the rank's strips + D2H gather of its f32 means and u8 image into pinned host memory",
        "host_sync": "each step" if a.sync_each else "after the K steps (frames streamed back to back)",
        # a frame's span, its trace's start to its sum's end: frames overlap under the frame
        # pipeline (a frame's sum runs beside the next frames' traces), so
        # this is longer than a step and no throughput follows from it
        "frame_span_ms": round(kernel_ms_max, 3),
        "segments_per_sample": round(total_segs / max(1.0, total_samples), 4),
        "scatters_per_sample": round(counts["scatters"] / max(1.0, counts["samples"]), 4),
        "trace_kernel_ms": round(trace_ms, 3),
        "trace_launches": launches,
        "trace_kernel_ms_per_launch": round(launch_ms, 3),
        "trace_kernel_ms_per_launch_events": round(launch_ms_events, 3),
        "trace_kernel_ms_min_max": [round(min(launch_log), 3), round(max(launch_log), 3)] if launch_log else None,
        "timing_source": f"HIP events around each of the {len(launch_log)} trace launches and {len(frame_log)} "
                         "renders of the K timed frames (fr_ctx_trace_log), averaged",
        "occupancy_wg_per_cu": stats[0]["occupancy"],
        "scene_kernel": {"specialised": jit["used"], "hiprtc_compiled": jit["compiled"],
                         "get_ms": round(jit["ms"], 1), "prepare_ms": round(prepare_ms, 1),
                         "what": "trace_kernel compiled for this scene's records (FR_FLAG_SCENE_JIT, jit.cpp), "
                                 "before the warm-up; same image bits as the compiled-in kernel"},
        "roofline": roof,
        "hbm_roofline": hbm,
    })
    if pmc:
        out["pmc"] = pmc
    out.update(check)
    if world == 1 and not a.no_cpu_baseline:
        out["cpu_baseline"] = cpu_baseline(a.cpu_budget)
        out["speedup_vs_cpu_baseline"] = round(value / out["cpu_baseline"]["value"], 1)
        try:
            out["cpu_baseline"]["c1"] = config_c1(ctx)
        except Exception as e:  # reported in the line; the headline above stands on its own
            out["cpu_baseline"]["c1"] = {"error": f"{type(e).__name__}: {e}"}
    frame.close()
    ctx.close()
    return out


def parse_args(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    # 20 frames (0.35 s of GPU time at N = 1): the frame pipeline's steady state, in which a
    # frame's sum runs beside the next frame's trace; the first and last
    # frames' sums are inside the timed region too
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-pmc", action="store_true", help="skip the rocprofv3 counter passes")
    ap.add_argument("--cpu-budget", type=float, default=12.0)
    ap.add_argument("--verify", action="store_true",
                    help="(kept for old command lines: every run now reports its frame hash, and N > 1 checks it "
                         "against the N = 1 frame)")
    ap.add_argument("--sync-each", action="store_true", help="wait for each frame's stats before the next")
    ap.add_argument("--no-scene-jit", action="store_true",
                    help="run the compiled-in trace kernel instead of the scene-specialised one (same image)")
    return ap.parse_args(argv)


def main():
    a = parse_args()
    plan = launch_plan(a.gpus)
    import torch

    import forma_rt as fr  # after torch, so one HIP runtime serves both

    out = run_mctx(a, plan, torch, fr) if plan["mode"] == "mctx" else run_rank(a, plan, torch, fr)
    if out is not None:
        print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
