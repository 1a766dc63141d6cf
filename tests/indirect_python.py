"""Independent pure-Python restatement of light.wgsl's `indirect_lit_ambient` (one bounce and
MULTIPLE_BOUNCES, light.wgsl:1263-1498) and `spatial_reuse` (indirect and EMISSIVE_LIT variants,
light.wgsl:1500-1684), with the ReSTIR helpers they call (merge_reservoir 175-179,
load_previous_spatial_reservoir 201-210, reservoir_lifetime 913-915, temporal_restir 937-952,
compute_jacobian 985-1004, env_brdf 890-908, sample_cosine_hemisphere 537-549, jittered_deferred_uv
1007-1017) and utils.wgsl (hash 15-24, random_float 26-28, coords_to_uv 37-39).

TEST INFRASTRUCTURE.  Written from the WGSL, not from oracle/hk_oracle.c or csrc/: it builds on
tests/direct_python.py (the walks, hit_info, select_light_candidate, the Bevy shading and the reservoir
packing, themselves restated from the WGSL and pinned bit-exact by test_direct_independent.py), with
the same scalar float32 conventions: left-to-right evaluation, dot = ((x x' + y y') +
z z'), normalize(v) = v * (1 / sqrt(dot)), mix(a, b, t) = a (1 - t) + b t, IEEE minNum / maxNum,
mat3 * v = (t v.x + b v.y) + n v.z, pow(x, 2) by multiplication with WGSL pow's domain (x < 0 -> NaN),
out-of-bounds textureLoad -> 0.  sin / cos come from the oracle library's pinned implementations
(hko_sin / hko_cos), as in direct_python.
"""
from __future__ import annotations

import math

import numpy as np

import direct_python as dp
from direct_python import F, F32_EPSILON, F32_MAX, GOLDEN_RATIO, INV_TAU, MAX_VARIANCE, PI, RAY_BIAS, U32_MAX

DONT_EXCLUDE = U32_MAX
DONT_SAMPLE_EMISSIVE = dp.DONT_SAMPLE_EMISSIVE
SPATIAL_REUSE_TAPS = 4
SPATIAL_VARIANCE_SAMPLE_THRESHOLD = 4


# ------------------------------------------------------------------ utils.wgsl
def hash_u32(value: int) -> int:
    m = 0xFFFFFFFF
    s = value & m
    s ^= 2747636419
    s = (s * 2654435769) & m
    s ^= s >> 16
    s = (s * 2654435769) & m
    s ^= s >> 16
    s = (s * 2654435769) & m
    return s


def random_float(value: int):
    return F(float(hash_u32(value))) / F(4294967295.0)


def coords_to_uv(c, size):
    return ((F(c[0]) + F(0.5)) / F(size[0]), (F(c[1]) + F(0.5)) / F(size[1]))


def pow2(x):
    """WGSL pow(x, 2.0): exp2(2 log2 x) domain — NaN for x < 0 or NaN — evaluated as x * x."""
    if not (x >= 0):
        return F(np.nan)
    return x * x


def length(a):
    return np.sqrt(dp.dot(a, a))


# ------------------------------------------------------------------ frame helpers
class Frame:
    """The per-frame inputs a pass reads: frame uniform fields (view.rs:105-123), the view, the lights,
    the G-buffer planes (deferred size) and the blue noise."""

    def __init__(self, fr: dict, gb: dict, noise: np.ndarray):
        self.fr, self.gb, self.noise = fr, gb, noise
        self.n = fr["number"]
        self.size = fr["size"]              # render (integrator) size s
        self.dsize = fr.get("deferred_size", fr["size"])  # G-buffer size S
        self.ratio = fr["ratio"]

    def jittered_uv(self, uv, amplitude=F(0.25)):
        j = -amplitude if (self.n & 1) == 0 else amplitude
        r = self.ratio - F(1.0)
        return tuple(uv[k] + (j * (F(1.0) / F(self.dsize[k]))) * r for k in range(2))

    def deferred_coords(self, uv):
        d = self.jittered_uv(uv)
        return dp.f2i(d[0] * F(self.dsize[0])), dp.f2i(d[1] * F(self.dsize[1]))

    def load(self, plane, c):
        """textureLoad: out-of-bounds reads return zero."""
        a = self.gb[plane]
        if 0 <= c[0] < a.shape[1] and 0 <= c[1] < a.shape[0]:
            return a[c[1], c[0]]
        return np.zeros(a.shape[2:], F)

    def blue_noise(self, x, y):
        """light.wgsl:1293-1297: texture frame % 16, nearest + repeat, fract(v + frame * phi)."""
        n = self.n
        nu = (F(x) + F(n) + F(0.5)) / F(64.0)
        nv = (F(y) + F(n) + F(0.5)) / F(64.0)
        tx, ty = int(math.floor(dp.fract(nu) * F(64.0))), int(math.floor(dp.fract(nv) * F(64.0)))
        texel = self.noise[n % 16, ty, tx]
        fn = F(n) * GOLDEN_RATIO
        return tuple(dp.fract(F(t) / F(255.0) + fn) for t in texel)

    def view_direction(self, position):
        """calculate_view, perspective branch (the example cameras are perspective)."""
        return dp.normalize(dp.sub(self.fr["view_position"], position[:3]))


def load_previous(buf, uv, size):
    """load_previous_reservoir / load_previous_spatial_reservoir (light.wgsl:181-190, 201-210)."""
    if abs(uv[0] - F(0.5)) < F(0.5) and abs(uv[1] - F(0.5)) < F(0.5):
        c = (dp.f2i(uv[0] * F(size[0])), dp.f2i(uv[1] * F(size[1])))
        return dp.unpack_reservoir(buf[c[0] + size[0] * c[1]])
    return dp.zero_reservoir()


def temporal_restir(r, s, w_new, max_count):
    dp.update_reservoir(r, s, w_new)
    m = F(max_count)
    if r["count"] > m:
        r["w_sum"] = r["w_sum"] * (m / r["count"])
        r["w2_sum"] = r["w2_sum"] * (m / r["count"])
        r["count"] = m


def merge_reservoir(r, other, p):
    count = r["count"]
    dp.update_reservoir(r, other, (p * other["w"]) * other["count"])
    r["count"] = count + other["count"]


def reservoir_variance(r):
    with np.errstate(all="ignore"):
        v = r["w2_sum"] / r["count"] - pow2(r["w_sum"] / r["count"])
        v = v if r["count"] < F(1.0) else v / r["count"]
    return dp.fmin(v, MAX_VARIANCE)


def compute_jacobian(q, r):
    """light.wgsl:985-1004; q = the neighbour's sample, r = the pixel's sample."""
    normal = q["sample_normal"]
    with np.errstate(all="ignore"):
        cos_phi_1 = abs(dp.dot(dp.normalize(dp.sub(r["visible_position"][:3], q["sample_position"][:3])), normal))
        cos_phi_2 = abs(dp.dot(dp.normalize(dp.sub(q["visible_position"][:3], q["sample_position"][:3])), normal))
        term_1 = cos_phi_1 / dp.fmax(F(0.0001), cos_phi_2)
        num = length(dp.sub(q["visible_position"][:3], q["sample_position"][:3]))
        num = num * num
        denom = length(dp.sub(r["visible_position"][:3], q["sample_position"][:3]))
        denom = denom * denom
        term_2 = num / dp.fmax(denom, F(0.0001))
        return dp.clamp(term_1 * term_2, 1.0, 50.0)


def env_brdf(sc, V, N, surface):
    """light.wgsl:890-908."""
    base, refl, rough = surface["base"], surface["reflectance"], surface["roughness"]
    metal, occl = surface["metallic"], surface["occlusion"]
    NdotV = dp.fmax(dp.dot(N, V), F(0.0001))
    f0s = ((F(0.16) * refl) * refl) * (F(1.0) - metal)
    F0 = (f0s + base[0] * metal, f0s + base[1] * metal, f0s + base[2] * metal)
    diffuse_color = dp.scale(base, F(1.0) - metal)
    da = dp.env_brdf_approx(sc, diffuse_color, F(1.0), NdotV)
    sa = dp.env_brdf_approx(sc, F0, rough, NdotV)
    return dp.scale(dp.add(da, sa), occl)


def sample_cosine_hemisphere(sc, rand):
    r = np.sqrt(rand[0])
    theta = (F(2.0) * PI) * rand[1]
    t = (r * sc.cos(theta), r * sc.sin(theta))
    z = np.sqrt(F(1.0) - (t[0] * t[0] + t[1] * t[1]))
    return (t[0], t[1], z), (F(2.0) * INV_TAU) * z


def _trace_bounce(sc, fm, counts, origin, direction):
    counts["top"] += 1
    hit = dp.traverse_top(sc, origin, direction, F32_MAX, F(0.0), DONT_EXCLUDE)
    return hit, dp.hit_info(sc, origin, direction, hit)


def _nee(sc, fm, counts, rand, position, normal, hit_instance, view_dir, surface):
    """The next-event part of a bounce (light.wgsl:1338-1367 / 1414-1441): returns the shaded radiance
    divided by the candidate pdf, or None when no shadow ray is cast."""
    fr = fm.fr
    cand, info = dp.select_light_candidate(sc, fr, rand, position, normal, hit_instance)
    counts["emitter"] += cand["emitter_rays"]
    sample_directional = cand["emissive"] == DONT_SAMPLE_EMISSIVE
    if not (dp.dot(cand["direction"], normal) > 0 and cand["p"] > 0):
        return None
    origin = dp.add(position, dp.scale(normal, RAY_BIAS))
    direction = cand["direction"]
    counts["top"] += 1
    hit = dp.traverse_top(sc, origin, direction, cand["max"], cand["min"], cand["emissive"])
    dp.occlude_hit_info(origin, direction, hit, info)
    in_radiance = dp.input_radiance(sc, fr, direction, info, sample_directional, cand["emissive"], False)
    with np.errstate(all="ignore"):
        out = dp.shading(sc, fr, view_dir, normal, direction, surface, in_radiance)
        return tuple(c / cand["p"] for c in out)


# ------------------------------------------------------------------ indirect_lit_ambient (light.wgsl:1263-1498)
def indirect_lit_ambient(sc, fm: Frame, bufs, x, y, counts):
    """One pixel; bufs: 'prev' (read), 'cur', 'prev_spatial', 'spatial' ((N, 16) u32 records),
    'variance' (H, W) f32, 'render' (H, W, 4) f32 (rounded to f16 on store)."""
    fr = fm.fr
    W, H = fm.size
    idx = x + W * y
    uv = coords_to_uv((x, y), fm.size)
    dc = fm.deferred_coords(uv)
    pd = fm.load("position", dc)
    position = (pd[0], pd[1], pd[2], F(1.0))
    depth = pd[3]
    s = dp.zero_reservoir()
    if fr["indirect_bounces"] == 0 or depth < F32_EPSILON:
        z = dp.pack_reservoir(dp.zero_reservoir())
        for b in ("cur", "spatial", "prev_spatial"):
            bufs[b][idx] = z
        bufs["variance"][y, x] = F(0.0)
        bufs["render"][y, x] = 0.0
        return
    normal = dp.normalize(tuple(fm.load("normal", dc)))
    im = fm.load("instance_material", dc)
    im_x, im_y = dp.f2u(im[0]), dp.f2u(im[1])
    velocity_uv = fm.load("velocity_uv", dc)
    s["random"] = fm.blue_noise(x, y)
    s["visible_position"] = (position[0], position[1], position[2], depth)
    s["visible_normal"] = normal
    s["visible_instance"] = im_x
    radiance = [F(0.0)] * 4
    pdf = F(0.0)
    if fr["indirect_bounces"] >= 2:  # MULTIPLE_BOUNCES pipeline (light.rs:663-666)
        bounce = dict(s)
        transport = (F(1.0), F(1.0), F(1.0))
        n = 0
        while n < fr["indirect_bounces"] and any(c > F(0.01) for c in transport):
            rs, rs_pdf = sample_cosine_hemisphere(sc, bounce["random"][:2])
            origin = dp.add(bounce["visible_position"][:3], dp.scale(bounce["visible_normal"], RAY_BIAS))
            direction = dp.basis_mul(dp.normal_basis(bounce["visible_normal"]), rs)
            hit, info = _trace_bounce(sc, fm, counts, origin, direction)
            if n == 0:
                s["sample_position"], s["sample_normal"], pdf = info["position"], info["normal"], rs_pdf
            bounce["sample_position"], bounce["sample_normal"] = info["position"], info["normal"]
            if hit["inst"] != U32_MAX:
                surface = dp.retreive_surface(sc, info["mat"])
                surface["roughness"] = F(1.0)
                sp3 = bounce["sample_position"][:3]
                view_dir = dp.normalize(dp.sub(bounce["visible_position"][:3], sp3))
                out = _nee(sc, fm, counts, bounce["random"], sp3, bounce["sample_normal"], info["inst"], view_dir,
                           surface)
                if out is not None:
                    with np.errstate(all="ignore"):
                        if n > 0:
                            out = (F(0.0),) * 3 if rs_pdf < F(0.01) else tuple(c / rs_pdf for c in out)
                        lum = dp.lum(out)
                        if lum > F(fr["max_indirect_luminance"]):
                            out = tuple((c * F(fr["max_indirect_luminance"])) / lum for c in out)
                    radiance = [radiance[k] + transport[k] * out[k] for k in range(3)] + [radiance[3] + F(1.0)]
                transport = dp.mul(transport, env_brdf(sc, view_dir, bounce["sample_normal"], surface))
                fnum = F(fr["number"]) * GOLDEN_RATIO
                bounce["random"] = tuple(dp.fract(c + fnum) for c in bounce["random"])
                bounce["visible_position"] = bounce["sample_position"]
                bounce["visible_normal"] = bounce["sample_normal"]
            else:
                amb = dp.input_radiance(sc, fr, direction, info, False, DONT_SAMPLE_EMISSIVE, True)
                radiance = [radiance[k] + transport[k] * amb[k] for k in range(3)] + [radiance[3] + F(0.0)]
                break
            n += 1
    else:
        rs, pdf = sample_cosine_hemisphere(sc, s["random"][:2])
        origin = dp.add(s["visible_position"][:3], dp.scale(s["visible_normal"], RAY_BIAS))
        direction = dp.basis_mul(dp.normal_basis(s["visible_normal"]), rs)
        hit, info = _trace_bounce(sc, fm, counts, origin, direction)
        s["sample_position"], s["sample_normal"] = info["position"], info["normal"]
        if hit["inst"] != U32_MAX:
            surface = dp.retreive_surface(sc, info["mat"])
            surface["roughness"] = F(1.0)
            sp3 = s["sample_position"][:3]
            view_dir = dp.normalize(dp.sub(s["visible_position"][:3], sp3))
            out = _nee(sc, fm, counts, s["random"], sp3, s["sample_normal"], info["inst"], view_dir, surface)
            if out is not None:
                radiance = [radiance[k] + out[k] for k in range(3)] + [radiance[3] + F(1.0)]
        else:
            amb = dp.input_radiance(sc, fr, direction, info, False, DONT_SAMPLE_EMISSIVE, True)
            radiance = [radiance[k] + amb[k] for k in range(3)] + [radiance[3] + F(0.0)]
    s["radiance"] = tuple(radiance)

    # ReSTIR: temporal (light.wgsl:1452-1497)
    juv = fm.jittered_uv(uv)
    previous_uv = (juv[0] - velocity_uv[0], juv[1] - velocity_uv[1])
    r = load_previous(bufs["prev"], previous_uv, fm.size)
    if not dp.check_previous_reservoir(r, s) and \
            abs(previous_uv[0] - F(0.5)) <= F(0.5) and abs(previous_uv[1] - F(0.5)) <= F(0.5):
        pc = (dp.f2i(previous_uv[0] * F(W)), dp.f2i(previous_uv[1] * F(H)))
        bufs["prev_spatial"][pc[0] + W * pc[1]] = dp.pack_reservoir(r)
    surface = dp.retreive_surface(sc, im_y)
    V = fm.view_direction(position)
    with np.errstate(all="ignore"):
        L = dp.normalize(dp.sub(s["sample_position"][:3], s["visible_position"][:3]))
        sample_radiance = dp.shading(sc, fr, V, s["visible_normal"], L, surface, s["radiance"])
        w_new = dp.lum(sample_radiance) / pdf if pdf > F(0.0) else F(0.0)
    temporal_restir(r, s, w_new, fr["max_temporal_reuse_count"])
    with np.errstate(all="ignore"):
        L = dp.normalize(dp.sub(r["sample_position"][:3], r["visible_position"][:3]))
        out = dp.shading(sc, fr, V, r["visible_normal"], L, surface, r["radiance"])
        total_lum = r["count"] * dp.lum(out)
        r["w"] = r["w_sum"] / total_lum if total_lum > F(0.0) else F(0.0)
    r["visible_position"] = s["visible_position"]
    r["visible_normal"] = s["visible_normal"]
    r["lifetime"] = r["lifetime"] + F(1.0)
    bufs["variance"][y, x] = reservoir_variance(r)
    if fr["temporal_reuse"]:
        bufs["cur"][idx] = dp.pack_reservoir(r)
    with np.errstate(all="ignore"):
        bufs["render"][y, x] = [dp.f16(out[0] * r["w"]), dp.f16(out[1] * r["w"]), dp.f16(out[2] * r["w"]), F(1.0)]


# ------------------------------------------------------------------ spatial_reuse (light.wgsl:1500-1684)
def spatial_reuse(sc, fm: Frame, bufs, x, y, emissive_lit):
    """One pixel; bufs: 'cur' (the temporal records this frame's temporal pass stored, read),
    'prev_spatial' (read), 'spatial' (written), 'variance', 'render'.  The workgroup-shared copies of
    light.wgsl:1500-1524 hold exactly the records / depths a global load returns (the pass writes neither),
    so every neighbour is read from the buffers."""
    fr = fm.fr
    W, H = fm.size
    count_n, reuse_range = (8, F(10.0)) if emissive_lit else (16, F(20.0))
    idx = x + W * y
    uv = coords_to_uv((x, y), fm.size)
    dc = fm.deferred_coords(uv)
    pd = fm.load("position", dc)
    position = (pd[0], pd[1], pd[2], F(1.0))
    depth = pd[3]
    r = dp.unpack_reservoir(bufs["cur"][idx])
    if depth < F32_EPSILON:
        bufs["spatial"][idx] = dp.pack_reservoir(r)
        bufs["render"][y, x] = 0.0
        return
    im = fm.load("instance_material", dc)
    velocity_uv = fm.load("velocity_uv", dc)
    surface = dp.retreive_surface(sc, dp.f2u(im[1]))
    use_spatial_variance = r["count"] <= F(SPATIAL_VARIANCE_SAMPLE_THRESHOLD)
    juv = fm.jittered_uv(uv)
    previous_uv = (juv[0] - velocity_uv[0], juv[1] - velocity_uv[1])
    q = dict(r)
    s = dict(q)
    lifetime_limit = F32_MAX if F(fr["max_reservoir_lifetime"]) <= F(1.0) else F(fr["max_reservoir_lifetime"])
    if r["lifetime"] <= lifetime_limit:
        r = load_previous(bufs["prev_spatial"], previous_uv, fm.size)
    V = fm.view_direction(position)
    with np.errstate(all="ignore"):
        if emissive_lit:
            merge_reservoir(r, q, dp.lum(q["radiance"][:3]))
        else:
            L = dp.normalize(dp.sub(s["sample_position"][:3], s["visible_position"][:3]))
            out = dp.shading(sc, fr, V, s["visible_normal"], L, surface, s["radiance"])
            merge_reservoir(r, q, dp.lum(out))
    r["visible_position"] = s["visible_position"]
    r["visible_normal"] = s["visible_normal"]
    rsum = ((s["random"][0] + s["random"][1]) + s["random"][2]) + s["random"][3]
    rf = random_float(fr["number"])
    for i in range(1, count_n + 1):
        px = F(6.283185307) * dp.fract((F(i) * GOLDEN_RATIO + rsum) + rf)
        py = np.sqrt(F(i) / F(count_n)) * reuse_range
        offset = (py * sc.cos(px), py * sc.sin(px))
        scx, scy = dp.f2i(offset[0] + F(x)), dp.f2i(offset[1] + F(y))
        suv = coords_to_uv((scx, scy), fm.size)
        sdc = fm.deferred_coords(suv)
        if suv[0] < F(0.0) or suv[1] < F(0.0) or suv[0] > F(1.0) or suv[1] > F(1.0):
            continue
        sample_depth = fm.load("position", sdc)[3]
        q = dp.unpack_reservoir(bufs["cur"][scx + W * scy])
        with np.errstate(all="ignore"):
            depth_ratio = depth / sample_depth
        if depth_ratio < F(0.9) or depth_ratio > F(1.1):
            continue
        normal_miss = dp.dot(s["visible_normal"], q["visible_normal"]) < F(0.866)
        if q["count"] < F32_EPSILON or normal_miss:
            continue
        with np.errstate(all="ignore"):
            sample_direction = dp.normalize(dp.sub(q["sample_position"][:3], s["visible_position"][:3]))
        if dp.dot(sample_direction, s["visible_normal"]) < F(0.0):
            continue
        # screen-space depth march (light.wgsl:1608-1628)
        tap_interval = dp.fmax(F(1.0), py / F(SPATIAL_REUSE_TAPS + 1))
        tap_count = dp.f2u(py / tap_interval)
        inv = F(1.0) / np.sqrt(offset[0] * offset[0] + offset[1] * offset[1])
        dirn = (offset[0] * inv, offset[1] * inv)
        occluded = False
        for j in range(1, tap_count + 1):
            tap_dist = F(j) * tap_interval
            tap_uv = (uv[0] + (tap_dist * dirn[0]) / F(W), uv[1] + (tap_dist * dirn[1]) / F(H))
            tap_depth = fm.load("position", fm.deferred_coords(tap_uv))[3]
            t = F(j) / F(tap_count + 1)
            ref_depth = depth * (F(1.0) - t) + sample_depth * t
            if tap_depth > ref_depth + F(0.00001):
                occluded = True
                break
        if occluded:
            continue
        jacobian = compute_jacobian(q, s) if q["sample_position"][3] > F(0.5) else F(1.0)
        with np.errstate(all="ignore"):
            if emissive_lit:
                merge_reservoir(r, q, dp.lum(q["radiance"][:3]) / jacobian)
            else:
                out = dp.shading(sc, fr, V, s["visible_normal"], sample_direction, surface, q["radiance"])
                merge_reservoir(r, q, dp.lum(out) / jacobian)
    m = F(fr["max_spatial_reuse_count"])
    if r["count"] > m:
        r["w_sum"] = r["w_sum"] * (m / r["count"])
        r["w2_sum"] = r["w2_sum"] * (m / r["count"])
        r["count"] = m
    with np.errstate(all="ignore"):
        L = dp.normalize(dp.sub(r["sample_position"][:3], s["visible_position"][:3]))
        out = dp.shading(sc, fr, V, s["visible_normal"], L, surface, r["radiance"])
        total_lum = r["count"] * (dp.lum(r["radiance"][:3]) if emissive_lit else dp.lum(out))
        r["w"] = r["w_sum"] / total_lum if total_lum > F(0.0) else F(0.0)
    r["lifetime"] = r["lifetime"] + F(1.0)
    bufs["spatial"][idx] = dp.pack_reservoir(r)
    if use_spatial_variance:
        bufs["variance"][y, x] = reservoir_variance(r)
    with np.errstate(all="ignore"):
        bufs["render"][y, x] = [dp.f16(r["w"] * out[0]), dp.f16(r["w"] * out[1]), dp.f16(r["w"] * out[2]), F(1.0)]
