"""bench.py's launch logic on CPU (no device): how `--gpus N` maps onto processes and
devices (bench.launch_plan), and the argument parser the driver's command lines use."""
import pytest

import bench


def test_single_gpu_default():
    p = bench.launch_plan(1, {})
    assert p == {"mode": "single", "rank": 0, "world": 1, "devices": [0]}


@pytest.mark.parametrize("n", [2, 4, 8])
def test_plain_command_drives_all_devices_in_one_process(n):
    p = bench.launch_plan(n, {})
    assert p["mode"] == "mctx" and p["world"] == 1 and p["devices"] == list(range(n))


@pytest.mark.parametrize("spec,n,devs", [("0,0", 2, [0, 0]), ("0,0,0,0,0,0,0,0", 8, [0] * 8), ("3", 1, [3]),
                                         (" 1, 0 ", 2, [1, 0])])
def test_rehearsal_devices(spec, n, devs):
    p = bench.launch_plan(n, {"FR_BENCH_DEVICES": spec})
    assert p["devices"] == devs
    assert p["mode"] == ("mctx" if n > 1 else "single")


@pytest.mark.parametrize("spec,n", [("0,0,0", 2), ("0", 2), ("-1,0", 2)])
def test_rehearsal_device_list_must_match(spec, n):
    with pytest.raises(SystemExit):
        bench.launch_plan(n, {"FR_BENCH_DEVICES": spec})


def test_torchrun_ranks():
    env = {"RANK": "3", "WORLD_SIZE": "4", "LOCAL_RANK": "3"}
    assert bench.launch_plan(4, env) == {"mode": "ranks", "rank": 3, "world": 4, "devices": [3]}
    # every rank on one device (rehearsal under the launcher)
    assert bench.launch_plan(4, dict(env, FR_BENCH_DEVICE="0"))["devices"] == [0]
    with pytest.raises(SystemExit):
        bench.launch_plan(8, env)  # --gpus disagrees with the launcher


def test_bad_gpu_count():
    with pytest.raises(SystemExit):
        bench.launch_plan(0, {})


def test_parse_args_driver_command_line():
    a = bench.parse_args(["--gpus", "8", "--steps", "5", "--warmup", "1"])
    assert (a.gpus, a.steps, a.warmup, a.no_scene_jit) == (8, 5, 1, False)
    a = bench.parse_args([])
    assert (a.gpus, a.steps, a.warmup) == (1, 20, 2)


def test_frame_hash_is_the_rehearsal_checksum():
    import numpy as np
    m = np.zeros((4, 5, 3), np.float32)
    assert bench.frame_hash(m) == bench.frame_hash(m.copy()) and len(bench.frame_hash(m)) == 16


def test_n_gt_1_line_checks_its_stitched_frame_against_n1():
    """The driver's SCALE lines (N = 2, 4, 8) check themselves: rank 0 stitches the shards'
    strips (bench.gather_frame) and compares them with the frame rendered whole on its device
    (bench.compare_with_n1): equal frames report frame_matches_n1 = true, and a frame whose
    one shard differs in one ulp of one channel reports false."""
    import numpy as np
    rng = np.random.default_rng(3)
    h, w, n = 40, 6, 4
    whole = rng.random((h, w, 3), dtype=np.float32)
    stitched = np.zeros_like(whole)
    for k in range(n):  # each shard's rows (8-row strips, k mod n), as gather_frame places them
        rows = bench.shard_rows(h, k, n)
        stitched[rows] = whole[rows]
    r = bench.compare_with_n1(stitched, whole)
    assert r["frame_matches_n1"] and r["frame_sha256_16"] == r["n1_frame_sha256_16"]
    bad = stitched.copy()
    y = bench.shard_rows(h, 3, n)[2]
    bad[y, 1, 2] = np.nextafter(bad[y, 1, 2], np.float32(2.0))
    r = bench.compare_with_n1(bad, whole)
    assert not r["frame_matches_n1"] and r["frame_sha256_16"] != r["n1_frame_sha256_16"]


def test_flop_model_counts_the_box_segment_term():
    """flops.h's constants as bench.py reads them: a box scene pays o * inv once per segment
    (3 flops, the fma slab form) on top of 22 per box test; a sphere scene
    pays a = dot(d, d) (5) instead."""
    c = bench.flop_constants()
    assert c["kFlopSegment"] == 3 and c["kFlopSegmentBox"] == 3 and c["kFlopTestBox"] == 22
    counts = {"segments": 10, "hits": 0, "scatters": 0, "samples": 0}
    box = bench.algorithmic_flops(c, counts, {"Box": 6}, 0)
    sph = bench.algorithmic_flops(c, counts, {"Sphere": 2}, 0)
    assert box == 10 * (3 + 3 + 6 * 22) + 10 * c["kFlopSky"]
    assert sph == 10 * (3 + 5 + 2 * 18) + 10 * c["kFlopSky"]
