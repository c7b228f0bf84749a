"""Every compiled variant of the inference kernel families that a model's shapes alone do not reach,
against a float64 torch reference, through the self-test entry points of include/kdlae.h
(every kernel libkdlae.so can launch is reached by some GPU test):

* implicit-GEMM family (gemm.hip): each entry of the four variant tables, read from the library
  (``kdlae_debug_gemm_variant``) so the cases track the tables — r01 ``conv_gemm_kernel`` (resident
  1x1, chunked 1x1 / 3x3 / 3x3x3, plain / PixelUnshuffle / PixelShuffle stores; forced with route 1,
  the production fallback for ld % 4 != 0 views), r02 ``gemm_res_kernel`` (with / without residual),
  ``gemm_chunk_kernel`` and the fused attention-output ``gemm_attn_in_kernel``; LayerNorm on A
  (in-register and from precomputed row statistics), ragged N / K / pixel tails, dilation 2;
* MDTA depthwise + Gram (mdta.hip): ring, sweep and generic kernels for every head width 16..128;
* training LayerNorm fallback kernels (train.hip ``ln_fwd_kernel`` / ``ln_bwd_kernel``);
* the 3x3x3 small-input conv (conv_small.hip ``conv_small_in_kernel<3, NTO>``).
"""
import ctypes

import pytest
import torch
import torch.nn.functional as F

from rethink_acoustic_image_enhancement_amd import _lib

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda", 0)
c_int64, c_int, c_void_p = ctypes.c_int64, ctypes.c_int, ctypes.c_void_p


class GemmDesc(ctypes.Structure):
    """kdlae_debug_gemm_desc (include/kdlae.h)."""
    _fields_ = [("A", c_void_p), ("lda", c_int),
                ("Bn", c_int), ("F", c_int), ("H", c_int), ("W", c_int),
                ("ksize", c_int), ("kt", c_int), ("dil", c_int), ("cg_per_tap", c_int), ("kgroups", c_int),
                ("Wp", c_void_p), ("w_img_stride", c_int64), ("ntiles", c_int), ("N", c_int),
                ("bias", c_void_p),
                ("out", c_void_p), ("ldo", c_int),
                ("R", c_void_p), ("ldr", c_int),
                ("ln", c_int), ("ln_C", c_int), ("relu", c_int), ("out_mode", c_int),
                ("stats", c_void_p),
                ("Wm", c_void_p), ("wm_img_stride", c_int64), ("bias_m", c_void_p), ("out1", c_void_p),
                ("ldo1", c_int),
                ("NT", c_int), ("KG", c_int), ("wpe", c_int), ("group_tiles", c_int), ("tiles_per_block", c_int),
                ("route", c_int)]


class GramDesc(ctypes.Structure):
    """kdlae_debug_gram_desc (include/kdlae.h)."""
    _fields_ = [("qkv", c_void_p), ("ld", c_int), ("wdw", c_void_p), ("bdw", c_void_p),
                ("v_out", c_void_p), ("ldv", c_int), ("partial", c_void_p), ("partial_floats", c_int64),
                ("reduced", c_void_p), ("zeros", c_void_p),
                ("C", c_int), ("heads", c_int), ("Bn", c_int), ("H", c_int), ("W", c_int), ("route", c_int)]


class LnDesc(ctypes.Structure):
    """kdlae_debug_ln_desc (include/kdlae.h)."""
    _fields_ = [("dir", c_int), ("x", c_void_p), ("ldx", c_int), ("w", c_void_p), ("b", c_void_p),
                ("C", c_int), ("P", c_int64), ("biasfree", c_int), ("y", c_void_p), ("ldy", c_int),
                ("stats", c_void_p), ("dy", c_void_p), ("ldd", c_int), ("R", c_void_p), ("ldr", c_int),
                ("dx", c_void_p), ("lddx", c_int), ("part", c_void_p), ("nblk", c_int), ("route", c_int)]


class SmallInDesc(ctypes.Structure):
    """kdlae_debug_small_in_desc (include/kdlae.h)."""
    _fields_ = [("inp", c_void_p), ("sb", c_int64), ("sc", c_int64), ("sy", c_int64), ("sx", c_int64),
                ("st", c_int64), ("in_sub", c_void_p),
                ("Cin", c_int), ("Cout", c_int), ("dil", c_int), ("kt", c_int), ("F", c_int),
                ("w", c_void_p), ("bias", c_void_p), ("out", c_void_p), ("ldo", c_int),
                ("Bn", c_int), ("H", c_int), ("W", c_int), ("vh", c_int), ("vw", c_int), ("relu", c_int)]


def _ptr(t):
    return None if t is None else t.data_ptr()


def _call(fn, desc_cls, **kw):
    d = desc_cls()
    for k, v in kw.items():
        setattr(d, k, v)
    _lib.check(getattr(_lib.lib(), fn)(ctypes.byref(d), None), fn)
    torch.cuda.synchronize()


def _rand(*shape, seed=0):
    g = torch.Generator(device="cpu").manual_seed(seed)
    return (torch.rand(*shape, generator=g, dtype=torch.float64) * 2 - 1).float().to(DEV)


def _close(got, ref, K, what=""):
    err = (got.double() - ref).abs().max().item()
    tol = 1e-5 * (ref.abs().max().item() + 1) * max(1.0, K ** 0.5) / 4
    assert err <= tol, f"{what} max |err| {err:.3e} > {tol:.3e}"


def _variants(family):
    out, v = [], (c_int * 7)()
    lib = _lib.lib()
    while lib.kdlae_debug_gemm_variant(family, len(out), v):
        out.append(tuple(v))
    return out


def pack_fragments(Wmat, ntiles, kgroups):
    """[N][K] -> the GEMM fragment order (runtime.h pack_fragments): element (l, e) of tile (t, g) is
    W(16 t + l % 16, 16 g + 4 (l / 16) + e); zero past N / K."""
    Wp = torch.zeros(ntiles * 16, kgroups * 16, dtype=torch.float32, device=DEV)
    Wp[:Wmat.shape[0], :Wmat.shape[1]] = Wmat
    return Wp.view(ntiles, 16, kgroups, 4, 4).permute(0, 2, 3, 1, 4).contiguous().view(-1)


def _ln_ref(x, mode):
    mu = x.mean(-1, keepdim=True)
    var = ((x - mu) ** 2).mean(-1, keepdim=True)
    return (x - mu) / torch.sqrt(var + 1e-5) if mode == 2 else x / torch.sqrt(var + 1e-5)


def _gemm_case(NT, KG, c3, out_mode, route, group_tiles=0, ntiles=None, with_r=False, ln=0, attn_in=False,
               seed=0, kchunks=1, dil=1, kt=1, relu=0):
    """One GEMM launch with the tile shape (NT, KG) forced, checked against float64 torch.
    group_tiles > 0: resident schedule (KG = kgroups); else ~kchunks chunks of KG k-groups."""
    Bn, Fr, H, W = 2, (3 if kt == 3 else 1), 10, 14
    HW = Fr * H * W
    if c3:
        cg = max(1, round(kchunks * KG / (9 * kt)))
        kgroups = 9 * kt * cg
        Cin = 16 * cg
    else:
        kgroups = KG if (group_tiles or attn_in) else KG * kchunks - 1   # ragged last k-chunk
        if ln and not (group_tiles or attn_in):
            kgroups = min(kgroups, 32)   # row statistics (ln_stats_kernel) cover C <= 512
        Cin = 16 * kgroups
    K = 16 * kgroups
    if ntiles is None:
        ntiles = 2 * NT + 1
    N = 16 * ntiles - (4 if out_mode == 2 else 0)   # PixelShuffle: a ragged last tile (N % 4 == 0)
    stats_path = ln and not attn_in and (kgroups > KG and not group_tiles)
    # route 1 runs on an ld % 4 != 0 view (the production fallback's case) unless LN needs row stats
    lda = Cin + (3 if route == 1 and not stats_path else 4)
    A = _rand(Bn, HW, lda, seed=seed)
    Wt = _rand(N, K, seed=seed + 1) / (K ** 0.5)
    bias = torch.zeros(16 * ntiles, device=DEV)
    bias[:N] = _rand(N, seed=seed + 2)
    Wp = pack_fragments(Wt, ntiles, kgroups)
    x = A[:, :, :Cin].double()
    if not c3:
        xa = x
        if attn_in:
            M = _rand(Bn, K, K, seed=seed + 5) / (K ** 0.5)
            bm = _rand(K, seed=seed + 6)
            Xr = _rand(Bn, HW, K + 4, seed=seed + 7)
            x1 = Xr[:, :, :K].double() + torch.einsum("bpk,bnk->bpn", x, M.double()) + bm.double()
            xa = x1
        if ln:
            xa = _ln_ref(xa, ln)
        ref = xa @ Wt.double().T + bias[:N].double()
        ref = ref.view(Bn * Fr, H, W, N).permute(0, 3, 1, 2)
    elif kt == 1:
        w4 = Wt.double().view(N, 3, 3, Cin).permute(0, 3, 1, 2)     # k = tap * Cin + c
        ref = F.conv2d(x.view(Bn, H, W, Cin).permute(0, 3, 1, 2), w4, bias[:N].double(), padding=dil, dilation=dil)
    else:
        w5 = Wt.double().view(N, 3, 3, 3, Cin).permute(0, 4, 1, 2, 3)
        ref = F.conv3d(x.view(Bn, Fr, H, W, Cin).permute(0, 4, 1, 2, 3), w5, bias[:N].double(),
                       padding=(1, dil, dil), dilation=(1, dil, dil))
        ref = ref.permute(0, 2, 1, 3, 4).reshape(Bn * Fr, N, H, W)
    if out_mode == 1:
        ref = F.pixel_unshuffle(ref, 2)
    elif out_mode == 2:
        ref = F.pixel_shuffle(ref, 2)
    Nout = ref.shape[1]
    ref = ref.permute(0, 2, 3, 1).reshape(-1, Nout)          # [Bn * Fr * Ho * Wo][Nout], NHWC
    ldo = Nout + 4
    R = None
    if with_r:                                               # residual in the output geometry
        R = _rand(ref.shape[0], ldo, seed=seed + 3)
        ref = ref + R[:, :Nout].double()
    if relu:
        ref = ref.clamp_min(0)
    out = torch.full((ref.shape[0], ldo), 7.0, device=DEV)
    stats = torch.empty(Bn * HW * 2, device=DEV)
    kw = dict(A=_ptr(A), lda=lda, Bn=Bn, F=Fr, H=H, W=W, ksize=3 if c3 else 1, kt=kt, dil=dil,
              cg_per_tap=cg if c3 else 0, kgroups=kgroups, Wp=_ptr(Wp), ntiles=ntiles, N=N, bias=_ptr(bias),
              out=_ptr(out), ldo=ldo, R=_ptr(R), ldr=ldo, ln=ln, ln_C=K, relu=relu, out_mode=out_mode,
              stats=_ptr(stats), NT=NT, KG=KG, wpe=2, group_tiles=group_tiles, route=route)
    if attn_in:
        Mp = torch.cat([pack_fragments(M[b], KG, KG) for b in range(Bn)])
        out1 = torch.full((Bn, HW, K + 4), 7.0, device=DEV)
        kw.update(Wm=_ptr(Mp), wm_img_stride=K * K, bias_m=_ptr(bm), out1=_ptr(out1), ldo1=K + 4,
                  R=_ptr(Xr), ldr=K + 4, group_tiles=ntiles)
    _call("kdlae_debug_gemm", GemmDesc, **kw)
    _close(out[:, :Nout], ref, K, "out")
    assert torch.all(out[:, Nout:] == 7.0), "wrote past N"
    if attn_in:
        _close(out1[:, :, :K], x1, K, "x1")
        assert torch.all(out1[:, :, K:] == 7.0)


def _resident_group(NT, KG):
    """group size for a resident 1x1 case: ragged chunks where the LDS budget (~150 KiB of split
    records, 3 KiB per tile and pair of k-groups) allows"""
    budget = 150 // (3 * ((KG + 1) // 2))
    return min(2 * NT - 1, max(NT, budget // NT * NT)) if NT > 1 else 1


# ------------------------------------------------------------------------------ r01 conv_gemm_kernel
CONV = _variants(0) if torch.cuda.is_available() else []


@pytest.mark.parametrize("v", CONV, ids=[f"nt{v[0]}_kg{v[1]}_c{v[2]}_o{v[3]}_pf{v[4]}_res{v[6]}" for v in CONV])
def test_conv_gemm_variant(v):
    """route 1: conv_gemm_kernel<NT, KG, CONV3, OUT, PF, WPE, RES>.  Resident 1x1 variants over two
    weight groups, alternately with a residual or a WithBias LN; chunked 1x1 over 3 k-chunks (ragged
    last) with BiasFree LN from row statistics, residual and ReLU on OUT 0; 3x3 over ~2 k-chunks at
    dilation 2 on OUT 0, with a residual in the output geometry on the shuffled stores."""
    NT, KG, c3, out_mode, pf, wpe, res = v
    i = CONV.index(v)
    if res:
        gt = _resident_group(NT, KG)
        _gemm_case(NT, KG, False, 0, 1, group_tiles=gt, ntiles=2 * gt - 1 if gt > 1 else 2, with_r=bool(i % 2),
                   ln=0 if i % 2 else 2, seed=i)
    elif c3:
        _gemm_case(NT, KG, True, out_mode, 1, kchunks=2, dil=2 if out_mode == 0 else 1, with_r=out_mode != 0,
                   seed=i)
    else:   # split pairs may not straddle k-chunks: an odd KG runs K in one chunk
        _gemm_case(NT, KG, False, out_mode, 1, kchunks=1 if KG % 2 else 3, ln=1 if out_mode == 0 else 0,
                   with_r=out_mode == 0, relu=1, seed=i)


# ------------------------------------------------------------------------------ r02 kernels
RES2 = _variants(1) if torch.cuda.is_available() else []


def _res2_hasr_ok(NT, KG, NCH):
    return NT * NCH <= 12 and NT * NCH * KG <= 72 and KG <= 8   # gemm.hip res2_hasr_ok


@pytest.mark.parametrize("v", RES2, ids=[f"nt{v[0]}_kg{v[1]}_nch{v[2]}" for v in RES2])
def test_gemm_res_variant(v):
    """gemm_res_kernel<NT, KG, NCH, 2, HASR, PF>: a group of (NCH - 1) NT + 1 tiles (ragged last chunk),
    two weight groups (the second one tile smaller), LN on A; with a residual where the variant has one."""
    NT, KG, NCH = v[:3]
    i = RES2.index(v)
    gt = (NCH - 1) * NT + 1
    _gemm_case(NT, KG, False, 0, 0, group_tiles=gt, ntiles=2 * gt - 1 if gt > 1 else 2, ln=1 + i % 2, seed=100 + i)
    if _res2_hasr_ok(NT, KG, NCH):
        _gemm_case(NT, KG, False, 0, 0, group_tiles=gt, ntiles=2 * gt - 1 if gt > 1 else 2, with_r=True,
                   seed=200 + i)


CHUNK2 = _variants(2) if torch.cuda.is_available() else []


@pytest.mark.parametrize("v", CHUNK2, ids=[f"nt{v[0]}_kg{v[1]}_c{v[2]}_o{v[3]}" for v in CHUNK2])
def test_gemm_chunk_variant(v):
    """gemm_chunk_kernel<NT, KG, CONV3, OUT, HASR>: 1x1 over 3 k-chunks (BiasFree LN from row
    statistics + ReLU on OUT 0) or 3x3 over ~2 (dilation 2 on OUT 0); the residual instance where it
    exists; one 3x3x3 (Conv3d) case."""
    NT, KG, c3, out_mode = v[:4]
    i = CHUNK2.index(v)
    if c3:
        _gemm_case(NT, KG, True, out_mode, 0, kchunks=2, dil=2 if out_mode == 0 else 1, with_r=out_mode != 0,
                   seed=300 + i)
        if (NT, KG, out_mode) == (2, 4, 0):
            _gemm_case(NT, KG, True, 0, 0, kchunks=7, kt=3, seed=350 + i)
    else:   # split pairs may not straddle k-chunks: an odd KG runs K in one chunk
        kch = 1 if KG % 2 else 3
        _gemm_case(NT, KG, False, out_mode, 0, kchunks=kch, ln=1 if out_mode == 0 else 0,
                   relu=1 if out_mode == 0 else 0, seed=300 + i)
        if out_mode == 0 and NT * KG < 36:
            _gemm_case(NT, KG, False, 0, 0, kchunks=kch, with_r=True, seed=400 + i)


ATTN = _variants(3) if torch.cuda.is_available() else []


@pytest.mark.parametrize("ln", [1, 2])
@pytest.mark.parametrize("v", ATTN, ids=[f"nt{v[0]}_kg{v[1]}_nch{v[2]}" for v in ATTN])
def test_gemm_attn_in_variant(v, ln):
    """gemm_attn_in_kernel<NT, KG, NCH>: x1 = x + M v + bias_m (per-image M) stored, and
    out = LN(x1) W^T + b over (NCH - 1) NT + 1 output tiles."""
    NT, KG, NCH = v[:3]
    _gemm_case(NT, KG, False, 0, 0, attn_in=True, ln=ln, ntiles=(NCH - 1) * NT + 1, seed=500 + ATTN.index(v))


def test_gemm_route_agreement_bits():
    """The production dispatch (r02 straight-line resident kernel) and the r01 kernel give the same
    bits on one aligned 1x1 problem with LN (both accumulate k-group-major, k-step-minor)."""
    Bn, H, W, KG, ntiles = 2, 16, 16, 3, 6
    K, N = 16 * KG, 16 * ntiles
    A = _rand(Bn, H * W, K, seed=9)
    Wp = pack_fragments(_rand(N, K, seed=10), ntiles, KG)
    outs = []
    for route in (0, 1):
        out = torch.zeros(Bn, H * W, N, device=DEV)
        _call("kdlae_debug_gemm", GemmDesc, A=_ptr(A), lda=K, Bn=Bn, F=1, H=H, W=W, ksize=1, kt=1, dil=1,
              kgroups=KG, Wp=_ptr(Wp), ntiles=ntiles, N=N, out=_ptr(out), ldo=N, ln=2, ln_C=K, NT=6, KG=KG,
              wpe=2, group_tiles=ntiles, route=route)
        outs.append(out)
    assert torch.equal(outs[0], outs[1])


# ------------------------------------------------------------------------------ MDTA Gram
@pytest.mark.parametrize("route", [0, 1, 2])
@pytest.mark.parametrize("ct", [1, 2, 3, 4, 5, 6, 7, 8])
def test_gram_variant(ct, route):
    """dwconv_gram_{ring,sweep,}_kernel<CT> + gram_reduce: v, the per-head Gram q k^T and the squared
    norms of the depthwise-convolved q, k against float64 torch (H = 40, W = 48: strips of 16)."""
    Bn, H, W, heads = 2, 40, 48, 1 if ct > 4 else 2
    Ch = 16 * ct
    C = Ch * heads
    ld = 3 * C + 4
    qkv = _rand(Bn, H, W, ld, seed=ct)
    wdw = _rand(9, 3 * C, seed=ct + 10)
    bdw = _rand(3 * C, seed=ct + 20)
    v_out = torch.full((Bn, H * W, C), 7.0, device=DEV)
    nsl = 64 * 8
    CT = ct
    sf = CT * CT * 256 + 2 * Ch
    partial = torch.empty(Bn * heads * nsl * sf, device=DEV)
    reduced = torch.empty(Bn * heads, sf, device=DEV)
    zeros = torch.zeros(64, device=DEV)
    _call("kdlae_debug_gram", GramDesc, qkv=_ptr(qkv), ld=ld, wdw=_ptr(wdw), bdw=_ptr(bdw), v_out=_ptr(v_out),
          ldv=C, partial=_ptr(partial), partial_floats=partial.numel(), reduced=_ptr(reduced), zeros=_ptr(zeros),
          C=C, heads=heads, Bn=Bn, H=H, W=W, route=route)
    x = qkv[..., :3 * C].double().permute(0, 3, 1, 2)
    w = wdw.double().T.reshape(3 * C, 1, 3, 3)
    y = F.conv2d(x, w, bdw.double(), padding=1, groups=3 * C)       # [Bn][3C][H][W]
    q, k, v = y[:, :C].flatten(2), y[:, C:2 * C].flatten(2), y[:, 2 * C:].flatten(2)
    _close(v_out, v.permute(0, 2, 1), 9, "v")
    for b in range(Bn):
        for h in range(heads):
            qh, kh = q[b, h * Ch:(h + 1) * Ch], k[b, h * Ch:(h + 1) * Ch]
            G = qh @ kh.T
            ref = torch.cat([G.view(CT, 4, 4, CT, 16).permute(0, 3, 1, 4, 2).reshape(-1),
                             (qh * qh).sum(1), (kh * kh).sum(1)])
            _close(reduced[b * heads + h], ref, H * W, f"gram b{b} h{h}")


def test_gram_generic_width():
    """W % 16 != 0: production dispatch itself takes the generic kernel (route 0 == route 2 bits)."""
    Bn, H, W, C = 1, 20, 20, 48
    ld = 3 * C
    qkv = _rand(Bn, H, W, ld, seed=77)
    wdw = _rand(9, 3 * C, seed=78)
    outs = []
    for route in (0, 2):
        partial = torch.empty(64 * (9 * 256 + 96), device=DEV)
        reduced = torch.empty(1, 9 * 256 + 96, device=DEV)
        v_out = torch.empty(Bn, H * W, C, device=DEV)
        _call("kdlae_debug_gram", GramDesc, qkv=_ptr(qkv), ld=ld, wdw=_ptr(wdw), v_out=_ptr(v_out), ldv=C,
              partial=_ptr(partial), partial_floats=partial.numel(), reduced=_ptr(reduced), C=C, heads=1,
              Bn=Bn, H=H, W=W, route=route)
        outs.append(reduced)
    assert torch.equal(outs[0], outs[1])


# ------------------------------------------------------------------------------ training LayerNorm
@pytest.mark.parametrize("biasfree", [0, 1])
@pytest.mark.parametrize("C", [48, 96, 192, 320])
@pytest.mark.parametrize("route", [0, 1])
def test_layernorm_variant(C, biasfree, route):
    """ln_fwd_kernel / ln_bwd_kernel<V> (route 1, the fallback for misaligned views) and the lane-group
    ln2 kernels (route 0): y, stats, dx = R + dLN(dy), and the summed weight / bias partials."""
    P, nblk = 1000, 37
    ld = C + (3 if route else 4)
    x = _rand(P, ld, seed=C)
    w = _rand(C, seed=C + 1)
    b = None if biasfree else _rand(C, seed=C + 2)
    y = torch.full((P, ld), 7.0, device=DEV)
    stats = torch.empty(P, 2, device=DEV)
    _call("kdlae_debug_ln", LnDesc, dir=0, x=_ptr(x), ldx=ld, w=_ptr(w), b=_ptr(b), C=C, P=P, biasfree=biasfree,
          y=_ptr(y), ldy=ld, stats=_ptr(stats), route=route)
    xd = x[:, :C].double().requires_grad_(True)
    wd = w.double().requires_grad_(True)
    bd = None if biasfree else b.double().requires_grad_(True)
    xn = _ln_ref(xd, 1 if biasfree else 2)
    yr = xn * wd + (0 if biasfree else bd)
    _close(y[:, :C], yr.detach(), C, "y")
    assert torch.all(y[:, C:] == 7.0)
    dy = _rand(P, ld, seed=C + 3)
    R = _rand(P, ld, seed=C + 4)
    dx = torch.full((P, ld), 7.0, device=DEV)
    part = torch.empty(nblk, C if biasfree else 2 * C, device=DEV)
    _call("kdlae_debug_ln", LnDesc, dir=1, x=_ptr(x), ldx=ld, w=_ptr(w), C=C, P=P, biasfree=biasfree,
          stats=_ptr(stats), dy=_ptr(dy), ldd=ld, R=_ptr(R), ldr=ld, dx=_ptr(dx), lddx=ld, part=_ptr(part),
          nblk=nblk, route=route)
    yr.backward(dy[:, :C].double())
    _close(dx[:, :C], R[:, :C].double() + xd.grad, C, "dx")
    _close(part[:, :C].sum(0), wd.grad, P, "dw")
    if not biasfree:
        _close(part[:, C:].sum(0), bd.grad, P, "db")


# ------------------------------------------------------------------------------ 3x3x3 small-input conv
@pytest.mark.parametrize("Cout", [32, 48, 64, 96, 128, 160])
def test_small_in_conv3d_variant(Cout):
    """conv_small_in_kernel<3, NTO>: Conv3d 1 -> Cout (3x3x3, padding 1, dilation 1 / 2 spatially) on a
    NCDHW view, with the ASDQE difference input (in - in_sub), a valid extent below H x W and ReLU."""
    Bn, Fr, H, W = 2, 4, 12, 20
    dil = 2 if Cout % 32 else 1
    inp = _rand(Bn, 1, Fr, H, W, seed=Cout)
    sub = _rand(Bn, 1, Fr, H, W, seed=Cout + 1)
    w = _rand(Cout, 1, 3, 3, 3, seed=Cout + 2)
    bias = _rand(Cout, seed=Cout + 3)
    vh, vw = H - 2, W - 3
    ldo = Cout + 4
    out = torch.full((Bn * Fr * H * W, ldo), 7.0, device=DEV)
    _call("kdlae_debug_small_in", SmallInDesc, inp=_ptr(inp), sb=Fr * H * W, sc=Fr * H * W, sy=W, sx=1, st=H * W,
          in_sub=_ptr(sub), Cin=1, Cout=Cout, dil=dil, kt=3, F=Fr, w=_ptr(w), bias=_ptr(bias), out=_ptr(out),
          ldo=ldo, Bn=Bn, H=H, W=W, vh=vh, vw=vw, relu=1)
    x = (inp - sub).double()
    x[..., vh:, :] = 0
    x[..., :, vw:] = 0
    ref = F.conv3d(x, w.double(), bias.double(), padding=(1, dil, dil), dilation=(1, dil, dil)).clamp_min(0)
    ref = ref.permute(0, 2, 3, 4, 1).reshape(-1, Cout)
    _close(out[:, :Cout], ref, 27, "out")
    assert torch.all(out[:, Cout:] == 7.0)
