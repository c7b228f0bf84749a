"""Every compiled variant of the training GEMM family (train_rows.hip, train_cols.hip, train.hip's
tiled kernels) against a float64 torch reference, through the self-test entry point
``kdlae_debug_tgemm`` (include/kdlae.h).  The training step reaches only the variants its shapes
select; these cases pick each template instance on purpose (every kernel libkdlae.so
can launch is reached by some GPU test):

* row-streaming kernel ``tgemm_rows_kernel<NT, HASR, VECC>``: NT 1..8 output tiles per block,
  with / without a residual (+ per-column scale), float4 or element stores (N % 4 != 0, or a
  misaligned C view), K % 16 != 0 with NaN in the ld pad columns (must not leak), batching;
* pixel-reduction kernel ``tgemm_cols_kernel<TM, TN>``: every wave tile shape, ragged pixel counts,
  batched channel slices;
* tiled kernels ``tgemm_lean_kernel<AKC, BNC, RM>`` (every operand layout, 64- and 128-row tiles)
  and ``tgemm_kernel<AM, BMODE, RM>`` (misaligned plain operands, and the implicit-im2col 3x3 conv
  forward / transposed conv / weight gradient, dilation 1 and 2, with split-K).
"""
import ctypes

import pytest
import torch
import torch.nn.functional as F

from rethink_acoustic_image_enhancement_amd import _lib

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda", 0)
c_int64, c_int, c_void_p = ctypes.c_int64, ctypes.c_int, ctypes.c_void_p


class TGemmDesc(ctypes.Structure):
    """kdlae_debug_tgemm_desc (include/kdlae.h)."""
    _fields_ = [("A", c_void_p), ("sam", c_int64), ("sak", c_int64), ("amode", c_int),
                ("B", c_void_p), ("sbk", c_int64), ("sbn", c_int64), ("bmode", c_int),
                ("C", c_void_p), ("scm", c_int64), ("scn", c_int64),
                ("bias", c_void_p),
                ("R", c_void_p), ("srm", c_int64), ("srn", c_int64),
                ("rs", c_void_p),
                ("M", c_int), ("N", c_int), ("K", c_int), ("nz1", c_int), ("nz2", c_int),
                ("bA1", c_int64), ("bA2", c_int64), ("bB1", c_int64), ("bB2", c_int64), ("bC1", c_int64),
                ("bC2", c_int64), ("bR1", c_int64), ("bR2", c_int64), ("brs1", c_int64), ("brs2", c_int64),
                ("Bn", c_int), ("H", c_int), ("W", c_int), ("Cg", c_int), ("dil", c_int),
                ("lda", c_int64), ("ldb", c_int64),
                ("partial", c_void_p), ("partial_floats", c_int64),
                ("route", c_int), ("c_pad_ok", c_int), ("F", c_int)]


def _ptr(t, off=0):
    return None if t is None else t.data_ptr() + 4 * off


def _run(**kw):
    d = TGemmDesc()
    d.nz1 = d.nz2 = 1
    d.dil = 1
    for k, v in kw.items():
        setattr(d, k, v)
    _lib.check(_lib.lib().kdlae_debug_tgemm(ctypes.byref(d), None), "kdlae_debug_tgemm")
    torch.cuda.synchronize()


def _rand(*shape, seed=0):
    g = torch.Generator(device="cpu").manual_seed(seed)
    return (torch.rand(*shape, generator=g, dtype=torch.float64) * 2 - 1).float().to(DEV)


def _close(got, ref, K):
    err = (got.double() - ref).abs().max().item()
    tol = 1e-5 * (ref.abs().max().item() + 1) * max(1.0, K ** 0.5) / 4
    assert err <= tol, f"max |err| {err:.3e} > {tol:.3e}"


# ---------------------------------------------------------------------------------------------- rows
ROWS = [(nt, hasr, vecc) for nt in (1, 2, 3, 4, 6, 8) for hasr in (False, True) for vecc in (True, False)
        if not (hasr and nt > 4)]


@pytest.mark.parametrize("nt,hasr,vecc", ROWS)
def test_rows_kernel_variant(nt, hasr, vecc):
    """C[z] = A[z] W^T (+ bias) (+ rs * R) with NT = N / 16 tiles (K = 40: 3 k-groups, 8 valid in the
    last, NaN in the A pads); element stores via N % 4 != 0 or, with a residual (which needs
    N % 4 == 0), via a C view one float off 16-byte alignment."""
    M, K, lda, z = 300, 40, 44, 2
    N = 16 * nt - (0 if (vecc or hasr) else 2)
    A = _rand(z, M, lda, seed=nt)
    A[:, :, K:] = float("nan")
    Wt = _rand(z, N, K, seed=nt + 10)                # B(k, n) = Wt[n, k]  (forward form)
    bias = _rand(N, seed=nt + 20)
    ldc = N + 4
    Cbuf = torch.full((z * M * ldc + 8,), 7.0, device=DEV)
    coff = 1 if (hasr and not vecc) else 0            # misaligned C view -> element stores
    R = _rand(z, M, ldc, seed=nt + 30) if hasr else None
    rs = _rand(z, N, seed=nt + 40) if hasr else None
    _run(A=_ptr(A), sam=lda, sak=1, B=_ptr(Wt), sbk=1, sbn=K, C=_ptr(Cbuf, coff), scm=ldc, scn=1,
         bias=_ptr(bias), R=_ptr(R), srm=ldc, srn=1, rs=_ptr(rs), M=M, N=N, K=K, nz1=z,
         bA1=M * lda, bB1=N * K, bC1=M * ldc, bR1=M * ldc, brs1=N, route=1)
    C = Cbuf[coff:coff + z * M * ldc].view(z, M, ldc)
    ref = torch.einsum("zmk,znk->zmn", A[:, :, :K].double(), Wt.double()) + bias.double()
    if hasr:
        ref = ref + rs.double()[:, None, :] * R[:, :, :N].double()
    _close(C[:, :, :N], ref, K)
    assert torch.all(C[:, :, N:] == 7.0), "wrote past N"


def test_rows_kernel_transposed_weights_and_private_pad():
    """dX form B(k, n) = W[k, n] (n-contiguous weights) with K % 4 != 0 and N % 4 != 0 writing whole
    quads into a private row pad (c_pad_ok): the pad must read 0."""
    M, K, N, lda, ldc = 513, 254, 127, 256, 128
    A = _rand(M, lda, seed=3)
    A[:, K:] = float("nan")
    W = _rand(K, N, seed=4)
    C = torch.full((M, ldc), 7.0, device=DEV)
    _run(A=_ptr(A), sam=lda, sak=1, B=_ptr(W), sbk=N, sbn=1, C=_ptr(C), scm=ldc, scn=1, M=M, N=N, K=K,
         route=1, c_pad_ok=1)
    _close(C[:, :N], A[:, :K].double() @ W.double(), K)
    assert torch.all(C[:, N:] == 0.0)


# ---------------------------------------------------------------------------------------------- cols
COLS = [(tm, tn) for tm in (2, 3, 4) for tn in (2, 3, 4) if (tm, tn) != (4, 4)]


@pytest.mark.parametrize("tm,tn", COLS)
def test_cols_kernel_variant(tm, tn):
    """dW[z] = dY[z]^T X[z] over a ragged pixel count; M = 16 tm and N = 16 tn channels select the
    wave tile (TM, TN) (4 x 4 runs as 4 x 2), batched over 2 images x 2 head slices."""
    Ch_m, Ch_n = 16 * tm - 3, 16 * tn - 1
    if (tm, tn) == (4, 2):
        Ch_m, Ch_n = 61, 64  # 4 x 4 tiles -> the 4 x 2 wave tile
    P, z1, z2 = 1000, 2, 2
    lda, ldb = 2 * Ch_m + 8, 2 * Ch_n + 4
    dY = _rand(z1, P, lda, seed=tm)
    X = _rand(z1, P, ldb, seed=tn + 50)
    C = torch.zeros(z1, z2, Ch_m, Ch_n, device=DEV)
    part = torch.empty(8 << 20, device=DEV)
    _run(A=_ptr(dY), sam=1, sak=lda, B=_ptr(X), sbk=ldb, sbn=1, C=_ptr(C), scm=Ch_n, scn=1,
         M=Ch_m, N=Ch_n, K=P, nz1=z1, nz2=z2, bA1=P * lda, bA2=Ch_m, bB1=P * ldb, bB2=Ch_n,
         bC1=z2 * Ch_m * Ch_n, bC2=Ch_m * Ch_n, partial=_ptr(part), partial_floats=part.numel(), route=2)
    for h in range(z2):
        a = dY[:, :, h * Ch_m:(h + 1) * Ch_m].double()
        b = X[:, :, h * Ch_n:(h + 1) * Ch_n].double()
        _close(C[:, h], torch.einsum("zpm,zpn->zmn", a, b), P)


# (cout, cin) -> the implicit instances the dispatch can pick: TM = 2 / 3 / 4, TN = 3 (cin 16) or 4 (cin 64; 2 beside TM 4)
COLS3D = [(16, 16), (48, 16), (64, 16), (32, 64), (48, 64), (64, 64)]


@pytest.mark.parametrize("cout,cin", COLS3D)
def test_cols_kernel_implicit_conv3d(cout, cin):
    """Conv3d 3x3x3 weight gradient with the implicit-im2col B (bmode 4): dW'[o][tap * cin + c] =
    sum_p dZ[p][o] X[p + off(tap)][c] with zero padding, against float64 unfold (B 2, F 3, 16 x 32, a
    pixel stride wider than cin)."""
    B_, F_, H_, W_ = 2, 3, 16, 32
    P, ldx, ldz = B_ * F_ * H_ * W_, cin + 4, cout
    X = _rand(B_, F_, H_, W_, ldx, seed=cin)
    dZ = _rand(P, ldz, seed=cout + 7)
    C = torch.zeros(cout, 27 * cin, device=DEV)
    part = torch.empty(8 << 20, device=DEV)
    _run(A=_ptr(dZ), sam=1, sak=ldz, B=_ptr(X), sbk=ldx, sbn=1, bmode=4, C=_ptr(C), scm=27 * cin, scn=1,
         M=cout, N=27 * cin, K=P, Bn=B_, F=F_, H=H_, W=W_, Cg=cin, partial=_ptr(part),
         partial_floats=part.numel(), route=2)
    xp = torch.nn.functional.pad(X[..., :cin].double().cpu(), (0, 0, 1, 1, 1, 1, 1, 1))  # pad W, H, F
    cols = torch.stack([xp[:, dt:dt + F_, dy:dy + H_, dx:dx + W_, :]
                        for dt in range(3) for dy in range(3) for dx in range(3)], dim=4)  # [B,F,H,W,27,cin]
    ref = dZ.double().cpu().t() @ cols.reshape(P, 27 * cin)
    _close(C, ref.to(DEV), P)


# ---------------------------------------------------------------------------------------------- tiled
LEAN = [(akc, bnc, rm) for akc in (True, False) for bnc in (True, False) for rm in (1, 2)]


@pytest.mark.parametrize("akc,bnc,rm", LEAN)
def test_tiled_lean_variant(akc, bnc, rm):
    """C = A B with A stored k- or m-contiguous and B n- or k-contiguous (all float4-aligned), 64-row
    tiles (small grid) or 128-row tiles (>= 512 tiles of 128 x 64)."""
    M = 66000 if rm == 2 else 1000
    N, K = 64, 72
    Am = _rand(M, K, seed=1)
    Bm = _rand(K, N, seed=2)
    A = Am if akc else Am.t().contiguous()
    B = Bm if bnc else Bm.t().contiguous()
    C = torch.zeros(M, N, device=DEV)
    _run(A=_ptr(A), sam=K if akc else 1, sak=1 if akc else M, B=_ptr(B), sbk=N if bnc else 1,
         sbn=1 if bnc else K, C=_ptr(C), scm=N, scn=1, M=M, N=N, K=K, route=3)
    _close(C, Am.double() @ Bm.double(), K)


@pytest.mark.parametrize("M", [777, 70000])
def test_tiled_generic_misaligned(M):
    """Plain operands with strides that rule out float4 loads (the scalar-load tiled kernel), 64- and
    128-row tiles."""
    N, K = 50, 41
    A = _rand(M, 43, seed=5)
    B = _rand(K, 53, seed=6)
    C = torch.zeros(M, 51, device=DEV)
    _run(A=_ptr(A), sam=43, sak=1, B=_ptr(B), sbk=53, sbn=1, C=_ptr(C), scm=51, scn=1, M=M, N=N, K=K, route=3)
    _close(C[:, :N], A[:, :K].double() @ B[:, :N].double(), K)


def _nhwc(x):
    return x.permute(0, 2, 3, 1).contiguous()


@pytest.mark.parametrize("dil", [1, 2])
@pytest.mark.parametrize("big", [False, True])
def test_tiled_conv3_forward_and_transposed(dil, big):
    """Implicit-im2col 3x3 conv (bmode 2) and its transposed conv (bmode 3) over NHWC views against
    torch conv2d / conv_transpose2d, dilation 1 and 2; `big` = a >= 512-tile grid (128-row tiles)."""
    Bn, H, W = (1, 256, 272) if big else (2, 20, 28)
    Cin, Cout = 8, 24
    x = _rand(Bn, Cin, H, W, seed=7)
    w = _rand(Cout, Cin, 3, 3, seed=8)
    bias = _rand(Cout, seed=9)
    xh = _nhwc(x)
    P = Bn * H * W
    y = torch.zeros(P, Cout, device=DEV)
    _run(A=_ptr(xh), amode=1, lda=Cin, Cg=Cin, B=_ptr(w), bmode=2, C=_ptr(y), scm=Cout, scn=1, bias=_ptr(bias),
         M=P, N=Cout, K=9 * Cin, Bn=Bn, H=H, W=W, dil=dil, route=3)
    ref = F.conv2d(x.double(), w.double(), bias.double(), padding=dil, dilation=dil)
    _close(y.view(Bn, H, W, Cout), _nhwc(ref), 9 * Cin)
    # transposed conv of dY (Cout channels) back to Cin
    dy = _rand(Bn, Cout, H, W, seed=10)
    dyh = _nhwc(dy)
    dx = torch.zeros(P, Cin, device=DEV)
    _run(A=_ptr(dyh), amode=1, lda=Cout, Cg=Cout, B=_ptr(w), bmode=3, C=_ptr(dx), scm=Cin, scn=1,
         M=P, N=Cin, K=9 * Cout, Bn=Bn, H=H, W=W, dil=dil, route=3)
    ref = F.conv_transpose2d(dy.double(), w.double(), padding=dil, dilation=dil)
    _close(dx.view(Bn, H, W, Cin), _nhwc(ref), 9 * Cout)


@pytest.mark.parametrize("dil", [1, 2])
def test_tiled_conv3_weight_gradient_split_k(dil):
    """dW[co][ci][t] = sum_p dY[p, co] X[p + off_t, ci] (bmode 1: B shifted per tap z2, 9 taps as the
    batch), split-K partials + the fixed-order reduce, against torch's conv2d weight gradient."""
    Bn, H, W, Cin, Cout = 2, 24, 40, 12, 20
    x = _rand(Bn, Cin, H, W, seed=11)
    dy = _rand(Bn, Cout, H, W, seed=12)
    xh, dyh = _nhwc(x), _nhwc(dy)
    P = Bn * H * W
    dw = torch.zeros(Cout, Cin, 3, 3, device=DEV)
    part = torch.empty(8 << 20, device=DEV)
    _run(A=_ptr(dyh), sam=1, sak=Cout, B=_ptr(xh), bmode=1, ldb=Cin, C=_ptr(dw), scm=Cin * 9, scn=9, bC2=1,
         nz2=9, M=Cout, N=Cin, K=P, Bn=Bn, H=H, W=W, dil=dil, partial=_ptr(part), partial_floats=part.numel(),
         route=3)
    ref = torch.nn.grad.conv2d_weight(x.double(), (Cout, Cin, 3, 3), dy.double(), padding=dil, dilation=dil)
    _close(dw, ref, P)


def test_engine_dispatch_routes_agree():
    """route 0 (the engine's policy) on a tall contraction equals the tiled kernel's result."""
    M, N, K = 70000, 96, 48
    A = _rand(M, K, seed=13)
    Wt = _rand(N, K, seed=14)
    C0 = torch.zeros(M, N, device=DEV)
    C3 = torch.zeros(M, N, device=DEV)
    for C, route in ((C0, 0), (C3, 3)):
        _run(A=_ptr(A), sam=K, sak=1, B=_ptr(Wt), sbk=1, sbn=K, C=_ptr(C), scm=N, scn=1, M=M, N=N, K=K, route=route)
    _close(C0, A.double() @ Wt.double().t(), K)
    _close(C3, A.double() @ Wt.double().t(), K)
