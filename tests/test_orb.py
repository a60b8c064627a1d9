"""Tiled ORB: oracle restatement checks (CPU) and bit-exact HIP parity (GPU).

Reference: /root/reference/orb.py:4-38 (tiling + cv2.ORB detect/compute).
OpenCV is absent, so the ORB internals are the OpenCV 4.x semantics restated in
oracle/orb.c (parity against OpenCV itself is unpinned);
here each stage of that restatement is checked against an independent
definition, and the GPU must equal the oracle bit for bit: keypoint
coordinates, size, angle, response, octave and all 256 descriptor bits.
"""
import os

import numpy as np
import pytest

import oracle
from conftest import ROOT

CIRCLE = [(0, 3), (1, 3), (2, 2), (3, 1), (3, 0), (3, -1), (2, -2), (1, -3), (0, -3), (-1, -3),
          (-2, -2), (-3, -1), (-3, 0), (-3, 1), (-2, 2), (-1, 3)]


def _frames(n=2, W=1280, H=720, seed=0):
    from slam355.synthetic import stereo_sequence

    L, R, _, _ = stereo_sequence(n, W, H, seed=seed)
    return L, R


# ----------------------------------------------------------------------------- CPU
def test_pattern_table_matches_kernel_include():
    pat = oracle.orb_pattern()
    inc = open(os.path.join(ROOT, "slam-1_amd", "csrc", "orb_pattern.inc")).read()
    body = inc[inc.index("{") + 1: inc.index("};")]
    vals = np.array([int(v) for v in body.replace("\n", " ").split(",") if v.strip()])
    assert np.array_equal(vals.reshape(256, 4), pat.astype(int))
    assert tuple(pat[0]) == (8, -3, 9, 5) and tuple(pat[1]) == (4, 2, 7, -12)


def test_level_tables():
    assert list(oracle.orb_level_budget(56)) == [12, 10, 8, 7, 6, 5, 4, 4]
    assert list(oracle.orb_level_budget(14)) == [3, 3, 2, 2, 1, 1, 1, 1]
    assert sum(oracle.orb_level_budget(200)) == 200
    lw, lh, sc = oracle.orb_level_sizes(192, 216)  # C2 patch (w, h)
    assert list(lw) == [192, 160, 133, 111, 93, 77, 64, 54]
    assert list(lh) == [216, 180, 150, 125, 104, 87, 72, 60]
    assert list(oracle.orb_umax()[:16]) == [15, 15, 15, 15, 14, 14, 14, 13, 13, 12, 11, 10, 9, 8, 6, 3]


def _resize_py(src, dw, dh):
    """INTER_LINEAR_EXACT restated independently (8-bit fixed point)."""
    sh, sw = src.shape

    def coeffs(dsize, ssize):
        scale = 1.0 / (dsize / ssize)
        out = []
        for d in range(dsize):
            f = scale * (d + 0.5) - 0.5
            i = int(np.floor(f))
            if i < 0 or ssize == 1:
                out.append((0, 0))
            elif i >= ssize - 1:
                out.append((ssize - 1, 0))
            else:
                out.append((i, int(np.rint((f - i) * 256.0))))
        return out
    cx, cy = coeffs(dw, sw), coeffs(dh, sh)
    s = src.astype(np.int64)
    out = np.zeros((dh, dw), np.uint8)
    for y, (yo, y1) in enumerate(cy):
        for x, (xo, x1) in enumerate(cx):
            h0 = (256 - x1) * s[yo, xo] + (x1 * s[yo, xo + 1] if x1 else 0)
            v = (256 - y1) * h0
            if y1:
                v += y1 * ((256 - x1) * s[yo + 1, xo] + (x1 * s[yo + 1, xo + 1] if x1 else 0))
            out[y, x] = min((v + 32768) >> 16, 255)
    return out


@pytest.mark.parametrize("sw,sh,dw,dh", [(192, 216, 160, 180), (40, 37, 33, 31), (9, 5, 9, 4),
                                         (7, 7, 12, 11)])
def test_resize_linear_exact_restatement(sw, sh, dw, dh):
    rng = np.random.default_rng(sw * dh)
    src = rng.integers(0, 256, (sh, sw), dtype=np.uint8)
    assert np.array_equal(oracle.resize_linear_exact(src, dw, dh), _resize_py(src, dw, dh))


def test_fast_score_is_max_threshold_still_corner():
    rng = np.random.default_rng(1)

    def corner(im, x, y, t):
        v = int(im[y, x])
        p = [int(im[y + dy, x + dx]) for dx, dy in CIRCLE]
        for cond in (lambda q: q < v - t, lambda q: q > v + t):
            m = [cond(q) for q in p] * 2
            if any(all(m[s:s + 9]) for s in range(16)):
                return True
        return False

    for trial in range(6):
        im = (rng.integers(0, 2, (20, 20)) * 190 + rng.integers(0, 50, (20, 20))).astype(np.uint8)
        sc = oracle.fast_score_map(im, 20)
        for y in range(3, 17):
            for x in range(3, 17):
                c = corner(im, x, y, 20)
                assert c == (sc[y, x] > 0)
                if c:
                    t = 20
                    while t < 255 and corner(im, x, y, t + 1):
                        t += 1
                    assert sc[y, x] == t


def test_gauss_blur7_restatement():
    """Float path of GaussianBlur(7x7, sigma 2): FMA chains; fma(a,b,c) in float32 is
    emulated exactly here as float32(double(a)*double(b) + double(c)) (the product
    is exact in double and the operands are small integers/kernel weights)."""
    k = oracle.gauss_kernel7().astype(np.float64)
    assert abs(k.sum() - 1) < 1e-6 and np.allclose(k, k[::-1])
    rng = np.random.default_rng(2)
    img = rng.integers(0, 256, (23, 29), dtype=np.uint8)
    h, w = img.shape
    idx = lambda i, n: i if 0 <= i < n else (-i if i < 0 else 2 * n - 2 - i)  # noqa: E731
    f32 = np.float32
    R = np.zeros((h, w), np.float32)
    for y in range(h):
        for x in range(w):
            s = f32(0)
            for t in range(7):
                s = f32(float(img[y, idx(x + t - 3, w)]) * k[t] + float(s))
            R[y, x] = s
    out = np.zeros_like(img)
    for y in range(h):
        for x in range(w):
            s = f32(float(R[y, x]) * k[3])
            for t in range(1, 4):
                a = f32(R[idx(y + t, h), x] + R[idx(y - t, h), x])
                s = f32(float(a) * k[3 + t] + float(s))
            out[y, x] = np.clip(np.rint(s), 0, 255)
    assert np.array_equal(oracle.gauss_blur7(img), out)


def test_oracle_orb_tiles_structure():
    L, _ = _frames(1, 640, 480, seed=3)
    kp, octv, desc = oracle.orb_tiles(L[0], 14)
    assert 0 < len(kp) <= 36 * 14 + 36 * 4
    assert desc.dtype == np.uint8 and desc.shape == (len(kp), 32)
    assert (kp[:, 0] >= 0).all() and (kp[:, 0] < 640).all() and (kp[:, 1] < 480).all()
    # size = 31 * 1.2^octave, angles in degrees
    assert np.allclose(kp[:, 2], 31 * np.float32(1.2) ** octv, rtol=1e-6)
    assert (kp[:, 3] >= 0).all() and (kp[:, 3] < 360).all()
    kp2, o2, d2 = oracle.orb_tiles(L[0], 14)
    assert np.array_equal(kp, kp2) and np.array_equal(desc, d2)


def test_fast_atan2_known_answers():
    """cv::fastAtan2 (degrees, [0, 360)): exact on the axes, and the 7th-order
    polynomial stays within 0.01 deg of atan2 on a 0.25-deg sweep (OpenCV's
    documented bound is 0.3 deg)."""
    f = oracle.lib().oracle_fast_atan2
    assert f(0.0, 1.0) == 0.0 and f(1.0, 0.0) == 90.0
    assert f(0.0, -1.0) == 180.0 and f(-1.0, 0.0) == 270.0
    # on the diagonal the polynomial gives (p1 + p3 + p5 + p7) * 180/pi = 44.99046
    d = (0.9997878412794807 - 0.3258083974640975 + 0.1555786518463281 - 0.04432655554792128)
    assert abs(f(1.0, 1.0) - d * 180 / np.pi) < 1e-4 and abs(f(1.0, 1.0) - 45.0) < 0.0096
    assert abs(f(-3.0, -3.0) - (180 + d * 180 / np.pi)) < 1e-4
    worst = 0.0
    for deg in np.arange(0, 360, 0.25):
        y, x = np.float32(np.sin(np.radians(deg)) * 37), np.float32(np.cos(np.radians(deg)) * 37)
        a = f(float(y), float(x))
        assert 0.0 <= a < 360.0 or (a == 360.0 and deg > 359)
        ref = np.degrees(np.arctan2(float(y), float(x))) % 360.0
        worst = max(worst, min(abs(a - ref), 360 - abs(a - ref)))
    assert worst < 0.01


def test_ic_umax_table():
    """The circular-patch row extents of ORB's IC angle for HALF_PATCH_SIZE 15
    (the table every ORB implementation derives: cvRound(sqrt(15^2 - v^2)) with
    the symmetric fix-up above 15/sqrt(2))."""
    assert oracle.orb_umax()[:16].tolist() == [15, 15, 15, 15, 14, 14, 14, 13, 13, 12, 11, 10, 9,
                                               8, 6, 3]


def _np_ic_angle(img, x, y):
    um = oracle.orb_umax()
    m10 = m01 = 0
    for v in range(-15, 16):
        d = um[abs(v)]
        row = img[y + v, x - d:x + d + 1].astype(np.int64)
        u = np.arange(-d, d + 1)
        m10 += int((u * row).sum())
        m01 += int(v * row.sum())
    return m01, m10


@pytest.mark.parametrize("theta", [0, 30, 90, 135, 200, 270, 333])
def test_ic_angle_known_answers(theta):
    """Intensity centroid of a linear ramp along theta points along theta; the
    oracle's moments equal an independent NumPy sum over the same disc."""
    h = w = 64
    yy, xx = np.mgrid[0:h, 0:w].astype(np.float64)
    t = np.radians(theta)
    img = np.clip(np.rint(128 + 3.0 * ((xx - 32) * np.cos(t) + (yy - 32) * np.sin(t))), 0,
                  255).astype(np.uint8)
    a = oracle.lib().oracle_ic_angle(_p(img), w, 32, 32, _p(oracle.orb_umax()))
    m01, m10 = _np_ic_angle(img, 32, 32)
    ref = np.degrees(np.arctan2(m01, m10)) % 360.0
    assert min(abs(a - ref), 360 - abs(a - ref)) < 0.01
    assert min(abs(a - theta), 360 - abs(a - theta)) < 0.5  # rounding of the ramp
    if theta % 90 == 0:
        assert a == float(theta)


def _p(a):
    return np.ascontiguousarray(a).ctypes.data_as(__import__("ctypes").c_void_p)


def _np_harris(img, x0, y0):
    im = img.astype(np.int64)
    a = b = c = 0
    for y in range(y0 - 3, y0 + 4):
        for x in range(x0 - 3, x0 + 4):
            ix = 2 * (im[y, x + 1] - im[y, x - 1]) + (im[y - 1, x + 1] - im[y - 1, x - 1]) + \
                (im[y + 1, x + 1] - im[y + 1, x - 1])
            iy = 2 * (im[y + 1, x] - im[y - 1, x]) + (im[y + 1, x - 1] - im[y - 1, x - 1]) + \
                (im[y + 1, x + 1] - im[y - 1, x + 1])
            a, b, c = a + ix * ix, b + iy * iy, c + ix * iy
    f = np.float32
    scale = f(1) / (f(4 * 7) * f(255))
    ssss = scale * scale * scale * scale
    fa, fb, fc = f(a), f(b), f(c)
    return (fa * fb - fc * fc - f(0.04) * (fa + fb) * (fa + fb)) * ssss


def test_harris_response_known_answers():
    """cv::ORB HarrisResponses (7x7 block, Sobel 3x3, k = 0.04, scale
    1/(4*7*255), applied as scale^4): an ideal 255-step edge through the block
    gives exactly -0.04 (2/7)^2 (a = 14 * 1020^2 = 2/7 of (4*7*255)^2, b = c = 0),
    a flat block 0, a quadrant corner > 0; contrast x2 gives response x16; and
    every value equals an independent NumPy restatement bit for bit."""
    h = oracle.lib().oracle_harris
    img = np.zeros((32, 32), np.uint8)
    img[:, 16:] = 255
    r = h(_p(img), 32, 16, 16)
    assert abs(r - (-0.04 * (2 / 7) ** 2)) < 1e-7
    assert np.float32(r) == _np_harris(img, 16, 16)
    assert h(_p(np.full((32, 32), 77, np.uint8)), 32, 16, 16) == 0.0
    q = np.zeros((32, 32), np.uint8)
    q[16:, 16:] = 60
    r1 = h(_p(q), 32, 16, 16)
    assert r1 > 0 and np.float32(r1) == _np_harris(q, 16, 16)
    r2 = h(_p(q * 2), 32, 16, 16)
    assert abs(r2 / r1 - 16.0) < 1e-5
    rng = np.random.default_rng(3)
    n = rng.integers(0, 256, (32, 32), dtype=np.uint8)
    for (x, y) in ((5, 5), (16, 9), (26, 26)):
        assert np.float32(h(_p(n), 32, x, y)) == _np_harris(n, x, y)


def _dot_grid(H=200, W=200, step=10, values=(255,)):
    img = np.zeros((H, W), np.uint8)
    for j, y in enumerate(range(5, H - 5, step)):
        for i, x in enumerate(range(5, W - 5, step)):
            img[y, x] = values[(i + j) % len(values)]
    return img


def test_retain_best_keeps_boundary_ties():
    """KeyPointsFilter::retainBest keeps every keypoint whose response equals
    the n-th best (nth_element + partition on >=): identical isolated dots all
    survive both cuts (FAST score to 2n, Harris to n) at octave 0 though the
    level budget is 4; with two contrasts the cut falls between the groups and
    every dot of the stronger group survives."""
    nl = oracle.orb_level_budget(20)
    assert nl[0] == 4
    img = _dot_grid()
    inside = [(x, y) for y in range(5, 195, 10) for x in range(5, 195, 10)
              if 31 <= x < 169 and 31 <= y < 169]
    kp, octv, _ = oracle.orb_tiles(img, 20, 1, 0, 0)
    k0 = kp[octv == 0]
    assert len(k0) == len(inside) > nl[0]
    assert len(set(k0[:, 4].tolist())) == 1  # one Harris response shared by all
    assert sorted(map(tuple, k0[:, :2].astype(int).tolist())) == sorted(inside)
    img2 = _dot_grid(values=(255, 128))
    kp, octv, _ = oracle.orb_tiles(img2, 20, 1, 0, 0)
    k0 = kp[octv == 0]
    strong = [(x, y) for (x, y) in inside if img2[y, x] == 255]
    assert sorted(map(tuple, k0[:, :2].astype(int).tolist())) == sorted(strong)


# ----------------------------------------------------------------------------- GPU
def _gpu_vs_oracle(imgs, max_kp, **tiling):
    import torch
    from slam355 import orb

    t = torch.from_numpy(np.ascontiguousarray(imgs)).cuda()
    kp, octv, desc, cnt = orb.orb_batch(t, max_kp, **tiling)
    torch.cuda.synchronize()
    kp, octv, desc, cnt = kp.cpu().numpy(), octv.cpu().numpy(), desc.cpu().numpy(), cnt.cpu().numpy()
    args = (tiling.get("overlap_div", 2), tiling.get("height_div", 5), tiling.get("width_div", 10))
    for b in range(len(imgs)):
        ek, eo, ed = oracle.orb_tiles(imgs[b], max_kp, *args)
        n = cnt[b]
        assert n == len(ek), (b, n, len(ek))
        assert np.array_equal(kp[b, :n].view(np.uint32), ek.view(np.uint32)), b  # bitwise floats
        assert np.array_equal(octv[b, :n], eo), b
        assert np.array_equal(desc[b, :n], ed), b
    return cnt


@pytest.mark.gpu
def test_gpu_orb_c2_frames_bit_exact():
    L, R = _frames(2, 1280, 720, seed=0)
    cnt = _gpu_vs_oracle(np.concatenate([L, R]), 56)
    assert (cnt > 900).all()


@pytest.mark.gpu
def test_gpu_orb_bench_config_bit_exact():
    """The headline bench's ORB input exactly: textured-corridor frames
    (bench.py seed 1000) at 1280x720 with 64 kp per tile (~2090 kp/frame):
    every keypoint, octave and descriptor bit vs the restatement."""
    from slam355.synthetic import corridor_sequence

    L, R, _, _ = corridor_sequence(4, 1280, 720, seed=1000, device="cuda", as_numpy=True)
    cnt = _gpu_vs_oracle(np.concatenate([L[:3], R[:2]]), 64)
    assert (cnt > 1900).all()


@pytest.mark.gpu
def test_gpu_orb_c1_and_reference_cap_bit_exact():
    L, R = _frames(1, 640, 480, seed=1)
    _gpu_vs_oracle(np.concatenate([L, R]), 14)
    _gpu_vs_oracle(L, 200)  # max_number_of_kp used by main.py:75


@pytest.mark.gpu
def test_gpu_orb_noise_flat_and_small_images():
    rng = np.random.default_rng(7)
    noise = rng.integers(0, 256, (2, 480, 640), dtype=np.uint8)  # many FAST candidates, ties
    flat = np.full((1, 480, 640), 128, np.uint8)                  # no corners at all
    blocks = (np.kron(rng.integers(0, 2, (1, 60, 80)), np.ones((1, 8, 8))) * 255).astype(np.uint8)
    cnt = _gpu_vs_oracle(np.concatenate([noise, flat, blocks]), 14)
    assert cnt[2] == 0
    # a size where the last tile row/column is clipped by the image bounds
    odd = rng.integers(0, 256, (1, 301, 517), dtype=np.uint8)
    _gpu_vs_oracle(odd, 20)


@pytest.mark.gpu
def test_gpu_orb_extraction_detect_single_patch():
    from slam355 import orb

    L, _ = _frames(1, 176, 144, seed=4)  # the whole image must fit one workgroup's LDS
    kps, des = orb.orb_extraction_detect(L[0], 100)
    ek, eo, ed = oracle.orb_tiles(L[0], 100, 1, 0, 0)
    assert len(ek) > 0
    assert len(kps) == len(ek)
    assert np.array_equal(np.array([k.pt for k in kps], np.float32), ek[:, :2])
    assert np.array_equal(des, ed)


@pytest.mark.gpu
def test_gpu_orb_retain_best_ties_match_oracle():
    from slam355 import orb

    for img in (_dot_grid(), _dot_grid(values=(255, 128))):
        kps, des = orb.orb_extraction_detect(img, 20)
        ek, eo, ed = oracle.orb_tiles(img, 20, 1, 0, 0)
        assert len(kps) == len(ek) > 20
        assert np.array_equal(np.array([k.pt for k in kps], np.float32), ek[:, :2])
        assert np.array_equal(des, ed)


@pytest.mark.gpu
def test_gpu_orb_whole_frames_global_levels():
    """cv2.ORB_create(n).detectAndCompute on a whole frame (bag_of_words.py:12,17):
    level images too large for LDS live in global ping-pong buffers."""
    from slam355 import orb

    L, R = _frames(1, 640, 480, seed=6)
    rng = np.random.default_rng(8)
    noise = rng.integers(0, 256, (1, 480, 640), dtype=np.uint8)
    for img, n in ((L[0], 100), (R[0], 500), (noise[0], 500)):
        kps, des = orb.orb_extraction_detect(img, n)
        ek, eo, ed = oracle.orb_tiles(img, n, 1, 0, 0)
        assert len(kps) == len(ek) > 0
        assert np.array_equal(np.array([k.pt for k in kps], np.float32), ek[:, :2])
        assert np.array_equal(des, ed)
    L2, _ = _frames(1, 1280, 720, seed=7)
    kps, des = orb.orb_extraction_detect(L2[0], 1000)
    ek, eo, ed = oracle.orb_tiles(L2[0], 1000, 1, 0, 0)
    assert len(kps) == len(ek) > 0 and np.array_equal(des, ed)


@pytest.mark.gpu
def test_gpu_orb_reference_api_shapes():
    from slam355 import orb

    L, _ = _frames(1, 640, 480, seed=5)
    kps, des = orb.orb_detector_using_tiles(L[0], max_number_of_kp=14)
    ek, eo, ed = oracle.orb_tiles(L[0], 14)
    assert des.shape == (len(kps), 32) and des.dtype == np.uint8
    assert [k.pt for k in kps] == [(float(a), float(b)) for a, b in ek[:, :2]]


@pytest.mark.gpu
def test_gpu_count_min_running_minimum():
    """slam_count_min (the Tracker's device-side overflow flag): the running
    minimum over successive count arrays, negative counts included."""
    import torch
    from slam355 import _lib
    from slam355.device import ptr

    dmin = torch.full((1,), 1 << 30, dtype=torch.int32, device="cuda")
    seen = 1 << 30
    rng = np.random.default_rng(3)
    for n in (1, 65, 300, 0):
        c = rng.integers(-5, 3000, n).astype(np.int32)
        _lib.call("slam_count_min", ptr(torch.from_numpy(c).cuda()) if n else None, n, ptr(dmin), None)
        seen = min([seen] + c.tolist())
        torch.cuda.synchronize()
        assert int(dmin.item()) == seen, n


@pytest.mark.gpu
def test_gpu_orb_lds_floor_keeps_results():
    """slam_orb_set_lds_floor (placement knob: one ORB workgroup per CU) changes
    where the workgroups run, never what they compute: bit-identical outputs."""
    import torch
    from slam355 import _lib, orb

    L, R = _frames(1, 1280, 720, seed=4)
    t = torch.from_numpy(np.ascontiguousarray(np.concatenate([L, R]))).cuda()
    ref = [x.cpu().numpy().copy() for x in orb.orb_batch(t, 64)]
    try:
        _lib.call("slam_orb_set_lds_floor", 82432)
        got = [x.cpu().numpy().copy() for x in orb.orb_batch(t, 64)]
    finally:
        _lib.call("slam_orb_set_lds_floor", 0)
    n = ref[3]
    assert np.array_equal(got[3], n)
    for b in range(len(n)):
        for a, e in zip(got[:3], ref[:3]):
            assert np.array_equal(a[b, :n[b]], e[b, :n[b]]), b
