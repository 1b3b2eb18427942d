"""TEST INFRASTRUCTURE ONLY -- numpy restatement of the reference's SSAO post-process.

Only tests/ may import this module, and only as the checker; the product path
(sphereflake-raytracer_amd/csrc/sf_post.hip) never calls it.

Restates, in IEEE binary32 with the shaders' operation order:
  noise texture     SSAO.cpp:144-164 (std::mt19937(12512), uniform_real_distribution<float>(-1, 1)
                    as libstdc++ implements it, glm 0.9.5 normalize(vec4))
  SSAO pass         Shaders/post_ssao.glsl:19-61
  blur passes       Shaders/post_ssao_blur.glsl:21-67 (x then y, SSAO.cpp:121-141)
  final composite   Shaders/post_final.glsl:15-28 (main.cpp:321-330)
with the GL state they run under (main.cpp:181-203, GLFramebufferObject.cpp:41-45, SSAO.cpp:166-174):
G-buffer textures RGBA32F NEAREST/CLAMP; pass targets RGBA8 LINEAR/CLAMP (every pass output
quantised to 8 bits); noise RGBA32F LINEAR/REPEAT. Texture filtering is modelled with the texel
coordinate snapped to 8 fractional bits (NEAREST floor, GL bilinear blend), and division by a uniform
or a per-tap scalar as multiplication by the correctly rounded reciprocal -- the same model the HIP
kernels implement. Parity against GL driver output is unpinned (no GL here); parity of the noise
texture is pinned bit for bit against the reference's own std::mt19937 path (sf_ssao_noise).
"""
from __future__ import annotations

import numpy as np

F = np.float32
NOISE = 64
OFFSET = (F(0.0), F(1.3846153846), F(3.2307692308))   # post_ssao_blur.glsl:9
WEIGHT = (F(0.2270270270), F(0.3162162162), F(0.0702702703))   # :10
DEFAULTS = dict(intensity=F(0.51), scale=F(3.28), bias=F(0.23), normal_threshold=F(2.47),
                depth_threshold=F(0.01))   # SSAO.cpp:50-55


# ----------------------------------------------------------------------------- noise texture

def mt19937_raw(seed: int, n: int) -> list[int]:
    mt = [0] * 624
    mt[0] = seed & 0xFFFFFFFF
    for i in range(1, 624):
        mt[i] = (1812433253 * (mt[i - 1] ^ (mt[i - 1] >> 30)) + i) & 0xFFFFFFFF
    out, pos = [], 624
    while len(out) < n:
        if pos == 624:
            for i in range(624):
                y = (mt[i] & 0x80000000) | (mt[(i + 1) % 624] & 0x7FFFFFFF)
                mt[i] = mt[(i + 397) % 624] ^ (y >> 1) ^ (0x9908B0DF if y & 1 else 0)
            pos = 0
        y = mt[pos]
        pos += 1
        y ^= y >> 11
        y ^= (y << 7) & 0x9D2C5680
        y ^= (y << 15) & 0xEFC60000
        y ^= y >> 18
        out.append(y & 0xFFFFFFFF)
    return out


def ssao_noise() -> np.ndarray:
    """[64*64, 4] float32: SSAO.cpp:150-164. libstdc++ uniform_real_distribution<float>(a, b) =
    generate_canonical<float, 24>(mt) * (b - a) + a, canonical = float(draw) / 2^32 (one 32-bit draw),
    clamped below 1; glm normalize(vec4) = x * (1 / sqrt(((x*x + y*y) + z*z) + w*w))."""
    raw = np.array(mt19937_raw(12512, NOISE * NOISE * 4), np.uint64)
    canon = raw.astype(np.float32) / F(4294967296.0)
    canon = np.where(canon >= F(1), np.nextafter(F(1), F(0)), canon).astype(np.float32)
    v = (canon * F(2) + F(-1)).reshape(-1, 4)
    x, y, z, w = v[:, 0], v[:, 1], v[:, 2], v[:, 3]
    sqr = x * x + y * y + z * z + w * w
    inv = F(1) / np.sqrt(sqr)
    return (v * inv[:, None]).astype(np.float32)


# ----------------------------------------------------------------------------- texture model

def _snap(x, lim):
    return np.rint(np.fmin(np.fmax(x, F(-2)), F(lim) + F(2)) * F(256))


def nearest(u, size: int):
    t = np.floor(_snap(u * F(size), size) * F(1 / 256)).astype(np.int64)
    return np.clip(t, 0, size - 1)


def linear(u, size: int):
    c = _snap(u * F(size) - F(0.5), size)
    f = np.floor(c * F(1 / 256))
    a = ((c - f * F(256)) * F(1 / 256)).astype(np.float32)
    i = f.astype(np.int64)
    return np.clip(i, 0, size - 1), np.clip(i + 1, 0, size - 1), a


def blend(t00, t10, t01, t11, a, b):
    w00 = (F(1) - a) * (F(1) - b)
    w10 = a * (F(1) - b)
    w01 = (F(1) - a) * b
    w11 = a * b
    return ((w00 * t00 + w10 * t10) + w01 * t01) + w11 * t11


def unorm(k):
    return k.astype(np.float32) / F(255)


def quant(x):
    return np.floor(np.fmin(np.fmax(x, F(0)), F(1)) * F(255) + F(0.5)).astype(np.uint8)


def sample_u8(t, u, v):
    h, w = t.shape
    x0, x1, a = linear(u, w)
    y0, y1, b = linear(v, h)
    return blend(unorm(t[y0, x0]), unorm(t[y0, x1]), unorm(t[y1, x0]), unorm(t[y1, x1]), a, b)


def sample_noise(noise, u, v):
    cs = np.rint((u * F(NOISE) - F(0.5)) * F(256))
    ct = np.rint((v * F(NOISE) - F(0.5)) * F(256))
    fs, ft = np.floor(cs * F(1 / 256)), np.floor(ct * F(1 / 256))
    a, b = (cs - fs * F(256)) * F(1 / 256), (ct - ft * F(256)) * F(1 / 256)
    x0, y0 = fs.astype(np.int64) & 63, ft.astype(np.int64) & 63
    x1, y1 = (x0 + 1) & 63, (y0 + 1) & 63
    t = noise.reshape(NOISE, NOISE, 4)
    return [blend(t[y0, x0, c], t[y0, x1, c], t[y1, x0, c], t[y1, x1, c], a, b) for c in (0, 1)]


# ----------------------------------------------------------------------------- passes

def _background(p):
    return (p[..., 0] * p[..., 0] + p[..., 1] * p[..., 1] + p[..., 2] * p[..., 2]) == F(0)


def ssao(pos4, nrm4, radius, downscale=1, intensity=DEFAULTS["intensity"], scale=DEFAULTS["scale"],
         bias=DEFAULTS["bias"], noise=None):
    """post_ssao.glsl over the (W/d, H/d) target; returns uint8 [ah, aw]."""
    H, W = pos4.shape[:2]
    aw, ah = W // downscale, H // downscale
    noise = ssao_noise() if noise is None else noise
    fx = (np.arange(aw, dtype=np.float32) + F(0.5))[None, :].repeat(ah, 0)
    fy = (np.arange(ah, dtype=np.float32) + F(0.5))[:, None].repeat(aw, 1)
    rcx, rcy = F(1) / F(aw), F(1) / F(ah)
    u, v = fx * rcx, fy * rcy
    tx, ty = nearest(u, W), nearest(v, H)
    p, n = pos4[ty, tx, :3], nrm4[ty, tx, :3]
    bg = _background(p)
    with np.errstate(all="ignore"):
        rad = F(radius) / np.sqrt(np.abs(p[..., 2]))
        nx, ny = sample_noise(noise, u * F(0.1), v * F(0.1))
        rx, ry = nx * F(2) - F(1), ny * F(2) - F(1)
        ln = np.sqrt(rx * rx + ry * ry)
        il = F(1) / ln
        rx, ry = rx * il, ry * il

        def occlude(ox, oy):
            sx, sy = nearest((fx + ox) * rcx, W), nearest((fy + oy) * rcy, H)
            s = pos4[sy, sx, :3]
            dx, dy, dz = s[..., 0] - p[..., 0], s[..., 1] - p[..., 1], s[..., 2] - p[..., 2]
            dist = np.sqrt(dx * dx + dy * dy + dz * dz)
            idt = F(1) / dist
            t = n[..., 0] * (dx * idt) + n[..., 1] * (dy * idt) + n[..., 2] * (dz * idt)
            m = t - F(bias)
            c = np.where(m > F(0), m, F(0)).astype(np.float32)
            return c * (F(1) / (F(1) + dist * dist * F(scale))) * F(intensity)

        ao = np.zeros_like(u)
        for kx, ky in ((1, 0), (-1, 0), (0, 1), (0, -1)):
            kx, ky = F(kx), F(ky)
            f = F(2) * (rx * kx + ry * ky)
            c1x, c1y = (kx - f * rx) * rad, (ky - f * ry) * rad
            c2x, c2y = c1x * F(0.707) - c1y * F(0.707), c1x * F(0.707) + c1y * F(0.707)
            ao = ao + occlude(c1x * F(0.25), c1y * F(0.25))
            ao = ao + occlude(c1x * F(0.75), c1y * F(0.75))
            ao = ao + occlude(c2x * F(0.5), c2y * F(0.5))
            ao = ao + occlude(c2x, c2y)
        ao = ao / F(16)
        out = quant(F(1) - ao)
    out[bg] = 0
    return out


def blur(pos4, nrm4, src, direction, normal_threshold=DEFAULTS["normal_threshold"],
         depth_threshold=DEFAULTS["depth_threshold"]):
    """post_ssao_blur.glsl over the W x H target; direction 0 = x, 1 = y. Returns uint8 [H, W]."""
    H, W = pos4.shape[:2]
    psx, psy = F(1) / F(W), F(1) / F(H)
    fx = (np.arange(W, dtype=np.float32) + F(0.5))[None, :].repeat(H, 0)
    fy = (np.arange(H, dtype=np.float32) + F(0.5))[:, None].repeat(W, 1)
    ux, uy = fx * psx, fy * psy
    tx, ty = nearest(ux, W), nearest(uy, H)
    p, n = pos4[ty, tx, :3], nrm4[ty, tx, :3]
    dx, dy = (F(0), F(1)) if direction else (F(1), F(0))
    color = np.zeros_like(ux)
    lo = np.zeros_like(ux)
    for k in (1, 2):
        ox, oy = dx * OFFSET[k] * psx, dy * OFFSET[k] * psy
        for side in (0, 1):
            sx, sy = (ux - ox, uy - oy) if side else (ux + ox, uy + oy)
            qx, qy = nearest(sx, W), nearest(sy, H)
            sp, sn = pos4[qy, qx, :3], nrm4[qy, qx, :3]
            d = n[..., 0] * sn[..., 0] + n[..., 1] * sn[..., 1] + n[..., 2] * sn[..., 2]
            acc = (d >= F(normal_threshold)) & (np.abs(sp[..., 2] - p[..., 2]) >= F(depth_threshold))
            color = np.where(acc, color + sample_u8(src, sx, sy) * WEIGHT[k], color).astype(np.float32)
            lo = np.where(acc, lo, lo + WEIGHT[k]).astype(np.float32)
    color = color + sample_u8(src, ux, uy) * (WEIGHT[0] + lo)
    return quant(color)


def final(pos4, ssao_tex, camera_position):
    """post_final.glsl; returns uint8 [H, W, 4]."""
    H, W = pos4.shape[:2]
    fx = (np.arange(W, dtype=np.float32) + F(0.5))[None, :].repeat(H, 0)
    fy = (np.arange(H, dtype=np.float32) + F(0.5))[:, None].repeat(W, 1)
    u, v = fx * (F(1) / F(W)), fy * (F(1) / F(H))
    p = pos4[nearest(v, H), nearest(u, W), :3]
    s = sample_u8(ssao_tex, u, v)
    cam = np.asarray(camera_position, np.float32)
    out = np.zeros((H, W, 4), np.uint8)
    for c in range(3):
        out[..., c] = quant((F(0.5) + F(0.5) * (p[..., c] + cam[c])) * s)
    out[..., 3] = 255
    out[_background(p)] = (0, 0, 0, 255)
    return out


def post_process(pos4, nrm4, camera_position, radius, downscale=1, **kw):
    """The full chain (SSAO.cpp:106-142 then main.cpp:321-330): returns (rgba, ao, blur_x, blur_y)."""
    sk = {k: kw[k] for k in ("intensity", "scale", "bias") if k in kw}
    bk = {k: kw[k] for k in ("normal_threshold", "depth_threshold") if k in kw}
    pos4 = np.ascontiguousarray(pos4, np.float32)
    nrm4 = np.ascontiguousarray(nrm4, np.float32)
    ao = ssao(pos4, nrm4, radius, downscale, **sk)
    bx = blur(pos4, nrm4, ao, 0, **bk)
    by = blur(pos4, nrm4, bx, 1, **bk)
    return final(pos4, by, camera_position), ao, bx, by
