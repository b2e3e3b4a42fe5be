"""Drive the host side of the C ABI under AddressSanitizer (tests/test_asan_host.py).

    LD_PRELOAD=<clang asan runtime> python tests/asan_host_calls.py <libsel_asan.so>

The library is the host-only ASan build (csrc/Makefile `asan`: no device code,
so nothing here may reach a kernel launch).  Calls every host-side entry point
that needs no GPU: the error paths of argument validation (null pointers, bad
descriptors and sizes, oversize job lists), the workspace / plan / geometry /
dispatch-decision functions over a sweep of shapes, the host-filled resampling
tap table, and the kernel-name writer with short buffers.  ctypes only (no
torch: the interpreter is not instrumented, only the library).  Prints "ok N"
with the number of calls; any ASan report aborts the process.
"""
import ctypes as C
import sys

lib = C.CDLL(sys.argv[1])
calls = 0


def fn(name, res, *args):
    f = getattr(lib, name)
    f.restype = res
    f.argtypes = list(args)
    return f


class ConvDesc(C.Structure):
    _fields_ = [("rows", C.c_int64), ("T", C.c_int32), ("C", C.c_int32), ("N", C.c_int32), ("K", C.c_int32),
                ("dil", C.c_int32), ("pad", C.c_int32), ("pad_mode", C.c_int32), ("in_elu", C.c_int32),
                ("bias_period", C.c_int32)]


class DconvDesc(C.Structure):
    _fields_ = [(n, C.c_int32) for n in ("B", "Tv", "Tvs", "ldx", "Tvo", "Tvalid", "ldo", "K", "q0", "S", "Cs", "Cg",
                                         "G", "So", "Ns", "Ng", "act")] + [("slope", C.c_float)]


class WgradJob(C.Structure):
    _fields_ = [("part", C.c_void_p), ("gw", C.c_void_p), ("gb", C.c_void_p), ("nw", C.c_int64),
                ("nsplit", C.c_int32), ("N", C.c_int32), ("bias_period", C.c_int32), ("kind", C.c_int32),
                ("cout", C.c_int32), ("cin", C.c_int32), ("k", C.c_int32), ("stride", C.c_int32)]


def call(f, *a):
    global calls
    calls += 1
    return f(*a)


P = C.c_void_p
I64, I32, SZ, F32 = C.c_int64, C.c_int, C.c_size_t, C.c_float

# library state
assert call(fn("sel_version", I32)) >= 1
tune = fn("sel_tune", I32, I32, I32)
for k in range(0, 64):
    old = call(tune, k, 7)
    assert call(tune, k, old) == 7
last = fn("sel_last_error", C.c_char_p)

# spectral argument validation and workspace sizes
stft = fn("sel_stft_mag_fwd", I32, P, I64, I64, I32, I32, I32, P, F32, P, P)
for args in ((None, 1, 100, 1000, 10, 100), (None, 0, 0, 0, 0, 0), (None, -1, -5, 1024, 0, 9999),
             (None, 2, 24000, 3000, 120, 600)):
    assert call(stft, *args, None, 1e-7, None, None) < 0
    assert call(last)
for name in ("sel_stft_bwd_workspace", "sel_stft_loss_workspace", "sel_logmel_bwd_workspace",
             "sel_mel_l1_workspace"):
    f = fn(name, SZ, I64, I64, I32, I32, I32)
    for B, T, n, h, w in ((1, 24000, 1024, 120, 600), (64, 24000, 2048, 300, 2048), (0, 0, 512, 50, 240),
                          (-3, 100, 0, 0, 0), (2, 7, 4096, 1, 4096)):
        call(f, B, T, n, h, w)
for name in ("sel_mag_pair_workspace", "sel_l1_workspace", "sel_add_noise_workspace"):
    f = fn(name, SZ, I64)
    for n in (0, 1, 7, 1 << 20, -5):
        call(f, n)
mell1 = fn("sel_mel_l1_fwd_grad", I32, P, P, I64, I64, I32, I32, I32, P, P, P, P, I32, F32, I32, P, P, P, SZ, P)
for args in ((1, 24000, 2048, 300, 2048, 80), (0, 24000, 2048, 300, 2048, 80), (2, 9000, 1024, 256, 1024, 0),
             (2, 9000, 1024, 256, 1024, 600), (2, 100, 1000, 10, 100, 80), (-1, 5, 256, 0, 0, 10)):
    B, T, n, h, w, nm = args
    assert call(mell1, None, None, B, T, n, h, w, None, None, None, None, nm, 1e-10, 0, None, None, None, 0, None) < 0
fin = fn("sel_stft_loss_finish", I32, P, I64, P, P)
assert call(fin, None, -1, None, None) < 0 and call(fin, None, 0, None, None) < 0

# conv descriptors: dispatch decisions, workspace plans, validation errors
kid = fn("sel_conv_fwd_kernel_id", I32, C.POINTER(ConvDesc), I32, I32, I32)
ws = fn("sel_conv_wgrad_workspace", SZ, C.POINTER(ConvDesc))
splits = fn("sel_resunit_wgrad_splits", I32, C.POINTER(ConvDesc), I32)
conv = fn("sel_conv_fwd", I32, C.POINTER(ConvDesc), I32, I32, P, P, P, P, P, P, P)
for (B, T, Cc, N, K, dil) in ((64, 24000, 32, 32, 7, 1), (64, 8000, 64, 64, 7, 9), (64, 2000, 128, 128, 7, 3),
                             (64, 400, 256, 256, 7, 9), (64, 400, 640, 256, 3, 1), (64, 24000, 1, 32, 7, 1),
                             (2, 40, 64, 64, 7, 9), (1, 1, 8, 8, 1, 1), (0, 10, 32, 32, 3, 1), (3, 5, 0, 4, 2, 1),
                             (2, 100, 33, 17, 9, 70), (1, 1 << 30, 64, 64, 7, 1)):
    for pad_mode in (0, 1):
        for elu in (0, 1):
            d = ConvDesc(B * T, T, Cc, N, K, dil, (K - 1) * dil, pad_mode, elu, N)
            for dt in (0, 1):
                call(kid, C.byref(d), dt, dt, elu)
                call(ws, C.byref(d))
                call(splits, C.byref(d), dt)
                rc = call(conv, C.byref(d), dt, dt, None, None, None, None, None, None, None)
                assert rc < 0 or B * T == 0, (B, T, Cc, N, K, dil, pad_mode, elu, dt, rc)
assert call(conv, None, 1, 1, None, None, None, None, None, None, None) < 0
bad = ConvDesc(-1, 0, -3, 0, 0, 0, -1, 5, 2, -1)
assert call(conv, C.byref(bad), 1, 1, None, None, None, None, None, None, None) < 0
bww = fn("sel_resunit_bwd_wgrad", I32, C.POINTER(ConvDesc), I32, P, P, P, P, P, P, P, P, I32, P)
d = ConvDesc(64 * 8000, 8000, 64, 64, 7, 3, 18, 0, 1, 64)
assert call(bww, C.byref(d), 1, None, None, None, None, None, None, None, None, 256, None) < 0

# batched weight-gradient reductions: bad job lists fail before any launch
finish = fn("sel_wgrad_finish_many", I32, P, I32, P)
assert call(finish, None, 3, None) < 0
jobs = (WgradJob * 30)()
for j in jobs:
    j.nsplit, j.N, j.nw = 0, 0, 0
assert call(finish, C.cast(jobs, P), 30, None) < 0
jobs[0].nsplit, jobs[0].N, jobs[0].nw = 1 << 20, 4, 16
assert call(finish, C.cast(jobs, P), 1, None) < 0

# batched discriminator weight-gradient reductions: bad job lists fail before any launch
dfin = fn("sel_dconv_wgrad_finish_many", I32, P, I32, P)
assert call(dfin, None, 2, None) < 0
assert call(dfin, None, 0, None) == 0


class DwgradJob(C.Structure):
    _fields_ = [(n, C.c_void_p) for n in ("part", "bpart", "v", "wg", "gw", "gg", "gb")] + \
               [(n, C.c_int32) for n in ("N", "Cg", "Kt", "stride", "pad", "G", "nsplit", "bsplit")]


djobs = (DwgradJob * 3)()
for jb in djobs:
    jb.N, jb.Cg, jb.Kt, jb.stride, jb.G, jb.nsplit = 4, 2, 3, 1, 1, 1
assert call(dfin, C.cast(djobs, P), 3, None) < 0  # null partials / outputs
djobs[0].part, djobs[0].gw, djobs[0].nsplit = 16, 16, 99
assert call(dfin, C.cast(djobs, P), 1, None) < 0  # nsplit past the presum bound
dpart = fn("sel_dconv_wgrad_partials", I32, P, I32, P, P, I32, I32, I32, I32, I32, P, P, P, P, P, P, SZ, P, P)
assert call(dpart, None, 1, None, None, 4, 2, 3, 1, 0, None, None, None, None, None, None, 0, None, None) < 0

# Adam over a tensor list: bad lists / constants fail before any launch
F64 = C.c_double
adam = fn("sel_adam_step_many", I32, P, I32, F64, F64, F64, F64, F64, F64, P)
assert call(adam, None, 3, 0.9, 0.999, 1e-8, 0.0, 1e-3, 0.5, None) < 0
assert call(adam, None, 0, 0.9, 0.999, 1e-8, 0.0, 1e-3, 0.5, None) == 0
assert call(adam, None, 0, 0.9, 0.999, 1e-8, 0.0, 1e-3, 0.0, None) < 0

# discriminator geometry, dispatch decision and kernel names (short buffers)
geo = fn("sel_dconv_geometry", I32, I32, I32, I32, C.POINTER(I32), C.POINTER(I32))
Kp, q0 = I32(), I32()
for Kt in range(1, 42):
    for s in range(1, 6):
        for pad in range(0, Kt + 1):
            call(geo, Kt, s, pad, C.byref(Kp), C.byref(q0))
call(geo, 0, 0, -1, C.byref(Kp), C.byref(q0))
dk = fn("sel_dconv_kernel", I32, C.POINTER(DconvDesc), I32, C.c_char_p, SZ)
dws = fn("sel_dconv_wgrad_workspace", SZ, C.POINTER(DconvDesc), I32)
for (B, T, S, Cg, G, Ng, K) in ((16, 9600, 3, 32, 1, 128, 2), (16, 24000, 1, 1, 1, 128, 15), (48, 400, 4, 64, 16, 256, 41),
                               (2, 10, 1, 1024, 1, 1024, 5), (0, 0, 0, 0, 0, 0, 0), (1, 3, 1, 1, 1, 1, 1)):
    d = DconvDesc(B, T, T + 4, S * Cg * G, T, T, Ng * G, K, -(K // 2), S, Cg * G if S > 1 else Cg, Cg, G, 1, Ng * G,
                  Ng, 1, 0.1)
    for dt in (0, 1):
        for cap in (0, 1, 5, 17, 256):
            buf = C.create_string_buffer(max(cap, 1))
            call(dk, C.byref(d), dt, buf if cap else None, cap)
        call(dws, C.byref(d), dt)

# resampling: plans for every common ratio and the host-filled tap table
plan = fn("sel_resample_plan", I32, I32, I32, I32, F32, C.POINTER(I32), C.POINTER(I32))
kern = fn("sel_resample_kernel", I32, I32, I32, I32, F32, P)
olen = fn("sel_resample_out_len", I64, I64, I32, I32)
ph, tp = I32(), I32()
for o, n in ((48000, 24000), (44100, 24000), (22050, 24000), (16000, 24000), (24000, 24000), (8000, 48000),
             (44100, 22050), (96000, 24000)):
    for width in (1, 6, 16):
        assert call(plan, o, n, width, 0.99, C.byref(ph), C.byref(tp)) == 0
        table = (C.c_float * (ph.value * tp.value))()
        assert call(kern, o, n, width, 0.99, C.cast(table, P)) == 0
        for L in (0, 1, 480, 123457):
            call(olen, L, o, n)
for args in ((0, 24000, 6, 0.99), (24000, 0, 6, 0.99), (-5, 24000, 6, 0.99), (48000, 24000, 0, 0.99),
             (48000, 24000, 6, 0.0), (48000, 24000, 6, 2.0)):
    call(plan, *args, C.byref(ph), C.byref(tp))
    assert call(kern, *args, None) < 0

# shape loss, RVQ and GAN-loss workspace sizes
sws = fn("sel_shape_loss_workspace", SZ, I64, I64, I32)
for r, T, w in ((64, 24000, 512), (1, 7, 8), (0, 0, 1), (3, 100, 0)):
    call(sws, r, T, w)
rws = fn("sel_rvq_workspace", SZ, I64, I32, I32)
for N, S, K in ((5120, 8, 1024), (1, 1, 1), (0, 0, 0), (100, 32, 4096)):
    call(rws, N, S, K)
call(fn("sel_gan_workspace", SZ))
print("ok", calls, flush=True)
