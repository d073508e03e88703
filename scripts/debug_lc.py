"""GPU bring-up aid: compare the kernel's stage dumps of one frame against the oracle."""
import ctypes as C
import sys
from pathlib import Path

import numpy as np
import torch

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
from jaadec_amd import native as N  # noqa: E402
from oracle import oracle as O  # noqa: E402


def oracle_stages(cfg, b, f=0):
    # overlap state entering frame f: run the oracle filterbank over frames < f
    ovs = np.zeros((2, 1024), np.float32)
    L = O.lib()
    L.orc_ms.argtypes = [C.c_void_p, C.c_int, C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p]
    L.orc_is.argtypes = [C.c_void_p, C.c_void_p, C.c_int, C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p]
    for ff in range(f + 1):
        iq = stage_iq(cfg, b, ff, L)
        if ff < f:
            for c in range(2):
                ic = b.ics[2 * ff + c]
                O.filterbank(int(ic["window_sequence"]), int(ic["window_shape"]), int(ic["window_shape_prev"]), iq[c], ovs[c])
    return finish(cfg, b, f, iq, ovs)


def stage_iq(cfg, b, f, L):
    iq = np.zeros((2, 1024), np.float32)
    for c in range(2):
        cf = 2 * f + c
        rs = np.array([b.ics[cf]["pns_state"]], np.uint32)
        rc = L.orc_dequant(b.ics[cf:cf + 1].ctypes.data, cfg.sf_index, b.q[cf].ctypes.data, b.sf[cf].ctypes.data,
                           b.cb[cf].ctypes.data, rs.ctypes.data, iq[c].ctypes.data)
        assert rc == 0
    iL = b.ics[2 * f:2 * f + 1]
    if (iL["flags"][0] & N.ICS_COMMON_WINDOW) and (iL["flags"][0] & N.ICS_MS_PRESENT):
        L.orc_ms(iL.ctypes.data, cfg.sf_index, b.cb[2 * f].ctypes.data, b.cb[2 * f + 1].ctypes.data,
                 b.ms_used[f].ctypes.data, iq[0].ctypes.data, iq[1].ctypes.data)
    L.orc_is(iL.ctypes.data, b.ics[2 * f + 1:2 * f + 2].ctypes.data, cfg.sf_index, b.cb[2 * f + 1].ctypes.data,
             b.sf[2 * f + 1].ctypes.data, b.ms_used[f].ctypes.data, iq[0].ctypes.data, iq[1].ctypes.data)
    return iq


def finish(cfg, b, f, iq, ovs):
    fftout = np.zeros((2, 1024), np.float32)
    outs = np.zeros((2, 1024), np.float32)
    for c in range(2):
        buf = O.imdct(iq[c])
        k = np.arange(512)
        re = np.where(k < 256, buf[(512 + 2 * k) % 2048], buf[(1024 + 2 * k - 512) % 2048])
        im = np.where(k < 256, -buf[(1536 + 2 * k) % 2048], buf[(2 * k - 512) % 2048])
        fftout[c, 0::2] = re
        fftout[c, 1::2] = im
        ov = ovs[c].copy()
        ic = b.ics[2 * f + c]
        outs[c] = O.filterbank(int(ic["window_sequence"]), int(ic["window_shape"]), int(ic["window_shape_prev"]), iq[c], ov)
    return iq, fftout, outs


def cmp(name, g, w):
    d = np.abs(g.astype(np.float64) - w.astype(np.float64))
    bad = np.flatnonzero(g.view(np.uint32) != w.view(np.uint32))
    print(f"{name}: {bad.size} differ, max|d|={d.max():.4g}, first bad idx {bad[:12]}")
    if bad.size:
        print("   got ", g[bad[:6]], "\n   want", w[bad[:6]])


def main():
    seq = int(sys.argv[1]) if len(sys.argv) > 1 else 2
    nfr = int(sys.argv[2]) if len(sys.argv) > 2 else 1
    dbgf = int(sys.argv[3]) if len(sys.argv) > 3 else 0
    p = N.synth_params(seq, n_streams=1, frames_per_stream=nfr)
    b = N.synth_batch(p)
    cfg = N.make_cfg()
    dbg = torch.zeros(6144 + 32 * 16, dtype=torch.float32, device="cuda")
    with N.Context(cfg, 1) as ctx:
        N.lib().jaad__debug_attach.argtypes = [C.c_void_p, C.c_void_p, C.c_int]
        N.lib().jaad__debug_attach(ctx.h, dbg.data_ptr(), dbgf)
        got = ctx.decode(b, N.PCM_FLOAT32)
    torch.cuda.synchronize()
    d = dbg.cpu().numpy()
    iq, fo, outs = oracle_stages(cfg, b, dbgf)
    print("ics", b.ics[:2])
    for c in range(2):
        cmp(f"spectrum ch{c}", d[1024 * c:1024 * (c + 1)], iq[c])
        cmp(f"fft/post ch{c}", d[2048 + 1024 * c:2048 + 1024 * (c + 1)], fo[c])
        cmp(f"out ch{c}", d[4096 + 1024 * c:4096 + 1024 * (c + 1)], outs[c])
    side = d[6144:].reshape(16, 4, 8)
    for f in range(min(nfr, 16)):
        print("frame", f, "gpu side L", side[f, 0, :7], "R", side[f, 1, :7])
        print("        host  L", [b.ics[2*f][k] for k in ("window_sequence","window_shape","window_shape_prev","max_sfb","flags")],
              "R", [b.ics[2*f+1][k] for k in ("window_sequence","window_shape","window_shape_prev","max_sfb","flags")])
    want = O.decode_batch(cfg, b, O.Streams(1), N.PCM_FLOAT32)
    gw = got.view(np.float32).reshape(nfr, -1); ww = want.view(np.float32).reshape(nfr, -1)
    print("frames equal:", [bool((gw[i].view(np.uint32) == ww[i].view(np.uint32)).all()) for i in range(nfr)])
    cmp("pcm f32", got.view(np.float32).reshape(-1), want.view(np.float32).reshape(-1))


if __name__ == "__main__":
    main()
