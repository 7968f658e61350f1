"""Pin the oracle (oracle/oracle.cpp) before trusting it.

1. The reference's own Vec3 known-answer tests, cpu_ray_tracer/primitives.rs:159-255
   (never compiled upstream; values verified to hold in IEEE f32).
2. Analytic known answers for utility.rs (reflect/refract/schlick), the shapes'
   hit() root cases (sphere.rs:23-51, plane.rs:24-44) and the build's box.
3. RNG vectors: splitmix64 (seed 0, published) and xoshiro128+ (state 1,2,3,4),
   checked against a pure-Python restatement of both.
"""
import math

import numpy as np
import pytest

from oracle import oracle_py as O
from oracle import scene_ref as S

f32 = np.float32


# ---- 1. primitives.rs:159-255 -------------------------------------------------

def test_length():  # :163-168
    a = (2.0, -3.0, -1.2)
    assert O.vec3(0, a)[0] == f32(14.440001)
    assert O.vec3(1, a)[0] == f32(3.8)


def test_dot():  # :170-179
    a, b = (1.0, 1.0, 1.0), (2.0, -3.0, -0.2)
    assert O.vec3(2, a, a)[0] == f32(3.0)
    assert O.vec3(2, b, b)[0] == f32(13.04)
    assert O.vec3(2, a, b)[0] == f32(-1.2)
    assert O.vec3(2, b, a)[0] == f32(-1.2)
    assert O.vec3(2, a, b)[0] == O.vec3(2, b, a)[0]


def test_cross():  # :181-189
    a, b = (1.0, 2.0, 3.0), (-3.0, -2.0, 1.0)
    assert O.vec3(3, a, a)[0] == 0.0
    assert O.vec3(3, b, b)[1] == 0.0
    assert O.vec3(3, a, b)[0] == 8.0
    assert O.vec3(3, b, a)[2] == -4.0


def test_addition():  # :191-204
    a, b = (1.0, 2.0, 3.0), (-3.0, -2.0, 1.0)
    assert list(O.vec3(4, a, b)) == [-2.0, 0.0, 4.0]
    assert list(O.vec3(4, a, b)) == list(O.vec3(4, b, a))


def test_subtraction():  # :206-219
    a, b = (1.0, 2.0, 3.0), (-3.0, -2.0, 1.0)
    assert list(O.vec3(5, a, b)) == [4.0, 4.0, 2.0]
    assert list(O.vec3(5, a, b)) == list(O.vec3(6, O.vec3(5, b, a), (-1.0, 0, 0)))


def test_multiplication():  # :221-241
    a, b = (1.0, 2.0, 3.0), (-3.0, -2.0, 1.0)
    assert list(O.vec3(6, a, (3.0, 0, 0))) == [3.0, 6.0, 9.0]
    assert list(O.vec3(7, a, b)) == [-3.0, -4.0, 3.0]


def test_division():  # :243-254
    assert list(O.vec3(8, (1.0, 2.0, 3.0), (2.0, 0, 0))) == [0.5, 1.0, 1.5]


# ---- 2. analytic known answers -------------------------------------------------

def test_unit_vector_and_reflect():
    u = O.vec3(9, (3.0, 0.0, 4.0))
    assert list(u) == [f32(0.6), 0.0, f32(0.8)]
    # reflect off the floor flips y only: v - 2*dot(v,n)*n
    assert list(O.vec3(10, (1.0, -1.0, 0.5), (0.0, 1.0, 0.0))) == [1.0, 1.0, 0.5]


def test_refract_normal_incidence_and_tir():
    ok, r = O.refract((0.0, -1.0, 0.0), (0.0, 1.0, 0.0), 1.0 / 1.3)
    assert ok and list(r) == [0.0, -1.0, 0.0]  # straight through
    ok, _ = O.refract((1.0, -0.05, 0.0), (0.0, 1.0, 0.0), 1.3)  # grazing, n1 > n2: total internal reflection
    assert not ok


def test_schlick_closed_form():
    r0 = ((1 - 1.3) / (1 + 1.3)) ** 2
    for c in (0.0, 0.25, 0.5, 1.0):
        want = r0 + (1 - r0) * (1 - c) ** 5
        assert abs(O.vec3(12, (c, 1.3, 0))[0] - want) < 2e-7
    assert O.vec3(12, (1.0, 1.3, 0))[0] == f32(f32(1 - f32(1.3)) / f32(1 + f32(1.3))) ** 2


def _sphere(c, r):
    return S.sphere(c, r, 0, (0.5, 0.5, 0.5), 0.0)


def test_sphere_outside_hit_near_root():
    best, rec = O.closest_hit([_sphere((0.0, 0.0, -5.0), 1.0)], (0, 0, 0), (0, 0, -1))
    assert best == 0 and rec[0] == 4.0 and list(rec[1:4]) == [0.0, 0.0, -4.0] and list(rec[4:]) == [0, 0, 1.0]


def test_sphere_inside_takes_far_root_with_outward_normal():
    best, rec = O.closest_hit([_sphere((0.0, 0.0, 0.0), 2.0)], (0, 0, 0), (0, 0, -1))
    assert best == 0 and rec[0] == 2.0 and list(rec[4:]) == [0, 0, -1.0]  # never flipped (sphere.rs:35,44)


def test_sphere_tangent_is_a_miss():
    best, _ = O.closest_hit([_sphere((1.0, 0.0, -5.0), 1.0)], (0, 0, 0), (0, 0, -1))
    assert best == -1  # discriminant > 0 is strict (sphere.rs:30)


def test_closest_wins_and_exact_ties_keep_the_first():
    a, b = _sphere((0, 0, -5.0), 1.0), _sphere((0, 0, -10.0), 1.0)
    assert O.closest_hit([b, a], (0, 0, 0), (0, 0, -1))[0] == 1
    assert O.closest_hit([a, a], (0, 0, 0), (0, 0, -1))[0] == 0  # t < t_max strict


def test_plane_gates_on_denominator_and_allows_negative_t():
    # plane.rs:26: `denom > t_min && denom < t_max` with denom = dot(orientation, d)
    p = S.plane((0.0, 0.0, -1.0), (0.0, 0.0, -1.0), (5.0, 5.0, 5.0), 0, (1, 1, 1), 0.0)
    best, rec = O.closest_hit([p], (0, 0, 0), (0, 0, -1))
    assert best == 0 and rec[0] == 1.0 and list(rec[4:]) == [0.0, 0.0, 1.0]
    best, rec = O.closest_hit([p], (0, 0, -2.0), (0, 0, -1))  # plane behind the origin: t = -1 accepted
    assert best == 0 and rec[0] == -1.0


def test_plane_failed_bounds_leave_stale_t_and_p():
    s = _sphere((0.0, 0.0, -5.0), 1.0)
    p = S.plane((0.0, 0.0, -2.0), (0.0, 0.0, -1.0), (0.1, 0.1, 0.1), 0, (1, 1, 1), 0.0)  # tiny plane
    best, rec = O.closest_hit([s, p], (0.5, 0.0, 0.0), (0, 0, -1))
    # the sphere wins, but the plane overwrote t and p before failing its bounds (plane.rs:28-29)
    assert best == 0 and rec[0] == 2.0 and list(rec[1:4]) == [0.5, 0.0, -2.0]
    assert rec[4] > 0  # normal is still the sphere's


def test_box_entry_exit_and_outward_normals():
    box = S.prim(S.AABB, 0, (1, 1, 1), 0.0, [-1, -1, -6, 1, 1, -4])
    best, rec = O.closest_hit([box], (0, 0, 0), (0, 0, -1))
    assert best == 0 and rec[0] == 4.0 and list(rec[4:]) == [0.0, 0.0, 1.0]
    best, rec = O.closest_hit([box], (0, 0, -5.0), (0, 0, -1))  # inside: exit face
    assert best == 0 and rec[0] == 1.0 and list(rec[4:]) == [0.0, 0.0, -1.0]
    assert O.closest_hit([box], (0, 2.0, 0), (0, 0, -1))[0] == -1


def test_obb_matches_aabb_for_identity_axes():
    obb = S.prim(S.OBB, 0, (1, 1, 1), 0.0, [0, 0, -5, 1, 0, 0, 0, 1, 0, 0, 0, 1, 1, 1, 1])
    best, rec = O.closest_hit([obb], (0.25, 0.5, 0), (0, 0, -1))
    assert best == 0 and rec[0] == 4.0 and list(rec[4:]) == [0.0, 0.0, 1.0]


def _tri(v0, v1, v2, material=0):
    return S.prim(S.TRIANGLE, material, (1, 1, 1), 0.0, list(v0) + list(v1) + list(v2))


def test_triangle_hit_barycentric_bounds_and_facing_normal():
    # triangle in z = -4; counter-clockwise seen from +z, so the winding normal is +z
    t = _tri((-1.0, -1.0, -4.0), (1.0, -1.0, -4.0), (0.0, 1.0, -4.0))
    best, rec = O.closest_hit([t], (0, 0, 0), (0, 0, -1))
    assert best == 0 and rec[0] == 4.0 and list(rec[1:4]) == [0.0, 0.0, -4.0] and list(rec[4:]) == [0, 0, 1.0]
    # from behind: the normal still faces the ray (double-faced meshes)
    best, rec = O.closest_hit([t], (0, 0, -8.0), (0, 0, 1))
    assert best == 0 and rec[0] == 4.0 and list(rec[4:]) == [0, 0, -1.0]
    # dielectric keeps the winding normal (inside/outside for refraction)
    best, rec = O.closest_hit([_tri((-1.0, -1.0, -4.0), (1.0, -1.0, -4.0), (0.0, 1.0, -4.0), 2)], (0, 0, -8.0), (0, 0, 1))
    assert best == 0 and list(rec[4:]) == [0, 0, 1.0]
    # outside the edges, behind t_min, and parallel rays miss
    assert O.closest_hit([t], (1.5, 0, 0), (0, 0, -1))[0] == -1
    assert O.closest_hit([t], (0, 0, -4.0005), (0, 0, 1))[0] == -1      # t = 0.0005 < t_min 0.001
    assert O.closest_hit([t], (0, 0, 0), (1, 0, 0))[0] == -1            # det = 0
    # a vertex and an edge point are inside (u, v >= 0, u + v <= 1 are closed)
    assert O.closest_hit([t], (-1.0, -1.0, 0), (0, 0, -1))[0] == 0
    assert O.closest_hit([t], (0.0, -1.0, 0), (0, 0, -1))[0] == 0


def test_triangle_list_order_and_ties():
    a = _tri((-1.0, -1.0, -4.0), (1.0, -1.0, -4.0), (0.0, 1.0, -4.0))
    b = _tri((-1.0, -1.0, -6.0), (1.0, -1.0, -6.0), (0.0, 1.0, -6.0))
    assert O.closest_hit([b, a], (0, 0, 0), (0, 0, -1))[0] == 1
    assert O.closest_hit([a, a], (0, 0, 0), (0, 0, -1))[0] == 0


def test_camera_new_basis():
    # camera.rs:24-60 at 2:1 aspect: w = +z, u = +x, v = +y, tan(30deg) half height
    c = O.camera_to_array(O.camera_new(200, 100))
    hh = f32(math.tan(f32(f32(60.0) * f32(3.14159265359) / f32(180.0)) / 2))
    # aspect, lens_radius = aperture/2, focus_dist stored 2.0, radius 5, rotation 0 (camera.rs:52-59)
    assert list(c[21:26]) == [2.0, f32(0.05), 2.0, 5.0, 0.0]
    assert list(c[12:15]) == [1.0, 0.0, 0.0] and list(c[18:21]) == [0.0, 0.0, 1.0]
    assert abs(c[10] - 2 * hh) < 1e-6  # vertical.y


# ---- 3. RNG vectors ---------------------------------------------------------------

M64 = (1 << 64) - 1


def _splitmix(x):
    x = (x + 0x9E3779B97F4A7C15) & M64
    z = x
    z = ((z ^ (z >> 30)) * 0xBF58476D1CE4E5B9) & M64
    z = ((z ^ (z >> 27)) * 0x94D049BB133111EB) & M64
    return x, z ^ (z >> 31)


def _rotl(v, k):
    return ((v << k) | (v >> (32 - k))) & 0xFFFFFFFF


def _xoshiro(s, n):
    s = list(s)
    out = []
    for _ in range(n):
        out.append((s[0] + s[3]) & 0xFFFFFFFF)
        t = (s[1] << 9) & 0xFFFFFFFF
        s[2] ^= s[0]
        s[3] ^= s[1]
        s[1] ^= s[2]
        s[0] ^= s[3]
        s[2] ^= t
        s[3] = _rotl(s[3], 11)
    return out


def test_published_vectors():
    assert _splitmix(0)[1] == 0xE220A8397B1DCDAF  # splitmix64, seed 0, first output
    # xoshiro128+ from state (1,2,3,4): s0 + s3 = 5, then state (7, 0, 1026, 12288) -> 12295, ...
    assert _xoshiro([1, 2, 3, 4], 2) == [5, 12295]


@pytest.mark.parametrize("seed,pixel,sample", [(0x5EED, 0, 0), (0x5EED, 2073599, 255), (7, 12345, 3), (0, 0, 0)])
def test_oracle_rng_matches_restatement(seed, pixel, sample):
    x = seed ^ ((pixel << 32) | sample)
    x, a = _splitmix(x)
    x, b = _splitmix(x)
    want = _xoshiro([a & 0xFFFFFFFF, a >> 32, b & 0xFFFFFFFF, b >> 32], 64)
    assert list(O.rng_stream(seed, pixel, sample, 64)) == want
