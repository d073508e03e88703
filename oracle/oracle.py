"""TEST INFRASTRUCTURE ONLY -- Python binding of the C restatement (oracle/jaad_oracle.c).

Imported only by tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg, always as the
checker / reported baseline, never as the measured or shipped path.  Parity status: see
oracle/jaad_oracle.h ("parity unpinned" by reference outputs; pinned by closed forms + fixtures).
"""
from __future__ import annotations

import ctypes as C
from pathlib import Path

import numpy as np

HERE = Path(__file__).resolve().parent
LIB_PATH = HERE / "liboracle.so"
_lib = None


def lib() -> C.CDLL:
    global _lib
    if _lib is None:
        if not LIB_PATH.exists():
            raise RuntimeError(f"{LIB_PATH} missing: run `python -m jaadec_amd.build`")
        L = C.CDLL(str(LIB_PATH))
        L.orc_fft.argtypes = [C.c_void_p, C.c_int, C.c_int]
        L.orc_fft.restype = None
        L.orc_imdct.argtypes = [C.c_void_p, C.c_void_p, C.c_int]
        L.orc_imdct.restype = None
        L.orc_filterbank.argtypes = [C.c_int, C.c_int, C.c_int, C.c_void_p, C.c_void_p, C.c_void_p]
        L.orc_filterbank.restype = None
        L.orc_dequant.argtypes = [C.c_void_p, C.c_int, C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p]
        L.orc_tns_spec.argtypes = [C.c_void_p, C.c_int, C.c_void_p, C.c_void_p]
        L.orc_tns_spec.restype = None
        L.orc_pcm_pack.argtypes = [C.c_void_p, C.c_int, C.c_int, C.c_uint32, C.c_void_p]
        L.orc_decode_batch.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p, C.c_size_t, C.c_uint32]
        L.orc_decode_batch_mt.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p, C.c_size_t, C.c_uint32,
                                          C.c_int]
        L.orc_stream_bytes.restype = C.c_size_t
        L.orc_streams_free.argtypes = [C.c_void_p, C.c_int]
        L.orc_streams_free.restype = None
        L.orc_sbr_dct4.argtypes = [C.c_void_p] * 4
        L.orc_sbr_dct4.restype = None
        L.orc_qmf_analysis_frame.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p, C.c_int]
        L.orc_qmf_analysis_frame.restype = None
        L.orc_qmf_synthesis_frame.argtypes = [C.c_void_p] * 4
        L.orc_qmf_synthesis_frame.restype = None
        L.orc_qmf_synthesis32_frame.argtypes = [C.c_void_p] * 4
        L.orc_qmf_synthesis32_frame.restype = None
        L.orc_sbr_table_info.argtypes = [C.c_void_p, C.c_int, C.c_void_p, C.c_void_p, C.c_void_p]
        L.jaad_write_frame.argtypes = [C.c_int, C.c_int] + [C.c_void_p] * 6 + [C.c_int, C.c_void_p, C.c_size_t]
        L.jaad_write_frame.restype = C.c_long
        L.jaad_write_frame_sbr.argtypes = ([C.c_int, C.c_int] + [C.c_void_p] * 6 + [C.c_int, C.c_void_p, C.c_void_p,
                                           C.c_void_p, C.c_size_t])
        L.jaad_write_frame_sbr.restype = C.c_long
        L.jaad_sbr_wstate_size.restype = C.c_size_t
        L.jaad_sbr_wstate_init.argtypes = [C.c_void_p, C.c_int, C.c_uint64]
        L.jaad_sbr_wstate_init.restype = None
        L.orc_sbr_res_tables.argtypes = [C.c_void_p, C.c_int, C.c_void_p, C.c_void_p]
        L.jaad_write_adts_header.argtypes = [C.c_int, C.c_int, C.c_size_t, C.c_void_p]
        L.jaad_write_frame_mc.argtypes = [C.c_int, C.c_int, C.c_void_p] + [C.c_void_p] * 6 + [C.c_void_p, C.c_size_t]
        L.jaad_write_frame_cce.restype = C.c_long
        L.jaad_write_frame_cce.argtypes = ([C.c_int, C.c_int, C.c_void_p] + [C.c_void_p] * 5 + [C.c_int] +
                                           [C.c_void_p] * 5 + [C.c_void_p, C.c_size_t])
        L.jaad_write_frame_mc.restype = C.c_long
        L.jaad_write_frame_mc_sbr.argtypes = ([C.c_int, C.c_int, C.c_void_p] + [C.c_void_p] * 6 + [C.c_void_p] * 2 +
                                              [C.c_void_p, C.c_size_t])
        L.jaad_write_frame_mc_sbr.restype = C.c_long
        L.jaad_write_frame_cce_sbr.argtypes = ([C.c_int, C.c_int, C.c_void_p] + [C.c_void_p] * 5 + [C.c_int] +
                                               [C.c_void_p] * 5 + [C.c_void_p] * 2 + [C.c_void_p, C.c_size_t])
        L.jaad_write_frame_cce_sbr.restype = C.c_long
        _lib = L
    return _lib


def fft(x: np.ndarray, forward: bool = False) -> np.ndarray:
    a = np.ascontiguousarray(np.stack([x.real, x.imag], -1).astype(np.float32))
    lib().orc_fft(a.ctypes.data, len(x), int(forward))
    return a[:, 0].astype(np.float64) + 1j * a[:, 1].astype(np.float64)


def imdct(spec: np.ndarray) -> np.ndarray:
    spec = np.ascontiguousarray(spec, np.float32)
    out = np.empty(2 * len(spec), np.float32)
    lib().orc_imdct(spec.ctypes.data, out.ctypes.data, 2 * len(spec))
    return out


def filterbank(seq: int, shape: int, shape_prev: int, spec: np.ndarray, overlap: np.ndarray) -> np.ndarray:
    spec = np.ascontiguousarray(spec, np.float32)
    out = np.empty(1024, np.float32)
    assert overlap.dtype == np.float32 and overlap.flags["C_CONTIGUOUS"]
    lib().orc_filterbank(seq, shape, shape_prev, spec.ctypes.data, out.ctypes.data, overlap.ctypes.data)
    return out


def pcm_pack(chans: list, flags: int = 0) -> bytes:
    arrs = [np.ascontiguousarray(c, np.float32) for c in chans]
    ptrs = (C.c_void_p * len(arrs))(*[a.ctypes.data for a in arrs])
    n = len(arrs[0])
    out = np.empty(n * len(arrs) * (4 if flags & 2 else 2), np.uint8)
    lib().orc_pcm_pack(ptrs, len(arrs), n, flags, out.ctypes.data)
    return out.tobytes()


def sbr_dct4(re: np.ndarray, im: np.ndarray):
    a, b = np.ascontiguousarray(re, np.float32), np.ascontiguousarray(im, np.float32)
    o_re, o_im = np.empty(32, np.float32), np.empty(32, np.float32)
    lib().orc_sbr_dct4(a.ctypes.data, b.ctypes.data, o_re.ctypes.data, o_im.ctypes.data)
    return o_re, o_im


class QmfAnalysis:
    """AnalysisFilterbank state (v[1280] ring + index) for frame-by-frame tests."""

    def __init__(self):
        self.v = np.zeros(1280, np.float32)
        self.idx = np.zeros(1, np.int32)

    def frame(self, x: np.ndarray, kx: int = 32) -> np.ndarray:
        x = np.ascontiguousarray(x, np.float32)
        X = np.zeros((32, 64, 2), np.float32)
        lib().orc_qmf_analysis_frame(self.v.ctypes.data, self.idx.ctypes.data, x.ctypes.data, X.ctypes.data, kx)
        return X


class QmfSynthesis:
    """SynthesisFilterbank64 state (v[2560] double ring + index)."""

    def __init__(self):
        self.v = np.zeros(2560, np.float32)
        self.idx = np.zeros(1, np.int32)

    def frame(self, X: np.ndarray) -> np.ndarray:
        X = np.ascontiguousarray(X, np.float32)
        out = np.empty(2048, np.float32)
        lib().orc_qmf_synthesis_frame(self.v.ctypes.data, self.idx.ctypes.data, X.ctypes.data, out.ctypes.data)
        return out


class QmfSynthesis32:
    """SynthesisFilterbank32 state (v[1280] double ring + index): downsampled SBR."""

    def __init__(self):
        self.v = np.zeros(1280, np.float32)
        self.idx = np.zeros(1, np.int32)

    def frame(self, X: np.ndarray) -> np.ndarray:
        X = np.ascontiguousarray(X, np.float32)
        out = np.empty(1024, np.float32)
        lib().orc_qmf_synthesis32_frame(self.v.ctypes.data, self.idx.ctypes.data, X.ctypes.data, out.ctypes.data)
        return out


def sbr_table_info(hdr, out_sf_index: int):
    """(info dict, f_master, f_table_lim) of FBT for a header (numpy record of SBR_HEADER_DTYPE)."""
    h = np.ascontiguousarray(np.array(hdr))
    info = np.zeros(12, np.int32)
    fm = np.zeros(64, np.int32)
    lim = np.zeros(64, np.int32)
    rc = lib().orc_sbr_table_info(h.ctypes.data, out_sf_index, info.ctypes.data, fm.ctypes.data, lim.ctypes.data)
    if rc:
        raise RuntimeError(f"orc_sbr_table_info failed: {rc}")
    keys = ["k0", "k2", "kx", "M", "N_master", "N_high", "N_low", "N_Q", "noPatches", "N_L", "gen_cnt", "max_src"]
    return dict(zip(keys, map(int, info))), fm, lim


def sbr_res_tables(hdr, out_sf_index: int):
    """(n[0], n[1], N_Q, N_high, N_low), f_table_res[2][64] of a header (calc_sbr_tables)."""
    h = np.ascontiguousarray(np.array(hdr))
    info = np.zeros(5, np.int32)
    ftr = np.zeros((2, 64), np.int32)
    rc = lib().orc_sbr_res_tables(h.ctypes.data, out_sf_index, info.ctypes.data, ftr.ctypes.data)
    if rc:
        raise RuntimeError(f"orc_sbr_res_tables failed: {rc}")
    return tuple(int(v) for v in info), ftr


class SbrWriter:
    """TEST WRITER state of one SBR stream (oracle/jaad_writer_sbr.c): tables of the current header
    and the previous frame's values its time-delta coding starts from."""

    def __init__(self, out_sf_index: int, seed: int = 1):
        self.buf = np.zeros(lib().jaad_sbr_wstate_size(), np.uint8)
        lib().jaad_sbr_wstate_init(self.buf.ctypes.data, out_sf_index, seed)


def write_frames(batch, sf_index: int, frames=None, extras: int = 0, sbr_writer: SbrWriter | None = None) -> list:
    """TEST WRITER: raw_data_block bytes of the given frames of a native.Batch (oracle/jaad_writer.c).
    extras bit 0 adds a DSE and a FIL fill element, bit 1 pulse data (both dropped by the parser).
    With sbr_writer, each frame's SBR record (batch.sbr) follows its channel element as a FIL."""
    nch = batch.nch
    frames = range(batch.n_frames) if frames is None else frames
    buf = np.zeros(16384, np.uint8)
    out = []
    for f in frames:
        cf = f * nch
        q = np.ascontiguousarray(batch.q[cf:cf + nch])
        sf = np.ascontiguousarray(batch.sf[cf:cf + nch])
        cb = np.ascontiguousarray(batch.cb[cf:cf + nch])
        ics = np.ascontiguousarray(batch.ics[cf:cf + nch])
        ms = np.ascontiguousarray(batch.ms_used[f]) if batch.ms_used is not None else np.zeros(2, np.uint64)
        tns = np.ascontiguousarray(batch.tns[cf:cf + nch]) if batch.tns is not None else None
        rec = np.ascontiguousarray(batch.sbr[f:f + 1]) if sbr_writer is not None else None
        n = lib().jaad_write_frame_sbr(sf_index, nch, q.ctypes.data, sf.ctypes.data, cb.ctypes.data, ics.ctypes.data,
                                       ms.ctypes.data, tns.ctypes.data if tns is not None else None, extras,
                                       rec.ctypes.data if rec is not None else None,
                                       sbr_writer.buf.ctypes.data if sbr_writer is not None else None,
                                       buf.ctypes.data, buf.nbytes)
        if n < 0:
            raise ValueError(f"frame {f} cannot be written")
        out.append(buf[:n].tobytes())
    return out


def write_frames_mc(batch, sf_index: int, ids, sbr_writers=None) -> list:
    """TEST WRITER: raw_data_blocks of a multichannel batch (native.mc_batch layout): the elements
    `ids` (0 SCE, 1 CPE, 3 LFE) in order, then END (jaad_write_frame_mc).  With sbr_writers (one
    SbrWriter or None per element), element k's SBR record batch.sbr[f, k] follows it as a FIL
    (jaad_write_frame_mc_sbr)."""
    nch = batch.nch
    ids_a = (C.c_int * len(ids))(*ids)
    buf = np.zeros(65536, np.uint8)
    out = []
    if sbr_writers is not None:
        states = (C.c_void_p * len(ids))(*[w.buf.ctypes.data if w is not None else None for w in sbr_writers])
        for f in range(batch.n_frames):
            cf = f * nch
            q = np.ascontiguousarray(batch.q[cf:cf + nch])
            sf = np.ascontiguousarray(batch.sf[cf:cf + nch])
            cb = np.ascontiguousarray(batch.cb[cf:cf + nch])
            ics = np.ascontiguousarray(batch.ics[cf:cf + nch])
            ms = np.ascontiguousarray(batch.ms_used[f]) if batch.ms_used is not None else np.zeros(2, np.uint64)
            tns = np.ascontiguousarray(batch.tns[cf:cf + nch]) if batch.tns is not None else None
            rec = np.ascontiguousarray(batch.sbr[f])
            n = lib().jaad_write_frame_mc_sbr(sf_index, len(ids), ids_a, q.ctypes.data, sf.ctypes.data, cb.ctypes.data,
                                              ics.ctypes.data, ms.ctypes.data, tns.ctypes.data if tns is not None else None,
                                              rec.ctypes.data, states, buf.ctypes.data, buf.nbytes)
            if n < 0:
                raise ValueError(f"frame {f} cannot be written")
            out.append(buf[:n].tobytes())
        return out
    for f in range(batch.n_frames):
        cf = f * nch
        q = np.ascontiguousarray(batch.q[cf:cf + nch])
        sf = np.ascontiguousarray(batch.sf[cf:cf + nch])
        cb = np.ascontiguousarray(batch.cb[cf:cf + nch])
        ics = np.ascontiguousarray(batch.ics[cf:cf + nch])
        ms = np.ascontiguousarray(batch.ms_used[f]) if batch.ms_used is not None else np.zeros(2, np.uint64)
        tns = np.ascontiguousarray(batch.tns[cf:cf + nch]) if batch.tns is not None else None
        n = lib().jaad_write_frame_mc(sf_index, len(ids), ids_a, q.ctypes.data, sf.ctypes.data, cb.ctypes.data,
                                      ics.ctypes.data, ms.ctypes.data, tns.ctypes.data if tns is not None else None,
                                      buf.ctypes.data, buf.nbytes)
        if n < 0:
            raise ValueError(f"frame {f} cannot be written")
        out.append(buf[:n].tobytes())
    return out


# jaad_cce_desc (oracle/jaad_writer.c): a coupling channel element to write
CCE_DESC_DTYPE = np.dtype([("ind_sw", "u1"), ("count", "u1"), ("domain", "u1"), ("sign", "u1"), ("scale", "u1"),
                           ("pair", "u1", (8,)), ("id", "u1", (8,)), ("chs", "u1", (8,)), ("pos", "u1"),
                           ("cge", "u1", (16,)), ("code", "i1", (16, 120))])


def write_frames_cce(batch, sf_index: int, ids, cces, sbr_writers=None) -> list:
    """TEST WRITER: raw_data_blocks of a (multichannel) batch with coupling channel elements:
    cces[f] = list of (desc CCE_DESC_DTYPE scalar, q [1024], sf [128], cb [128], ics ICS_DTYPE scalar)
    written before channel element desc["pos"] (jaad_write_frame_cce); with sbr_writers (one SbrWriter
    or None per element) each element's SBR record (batch.sbr [frame] or [frame][element]) follows it."""
    nch = batch.nch
    ids_a = (C.c_int * len(ids))(*ids)
    states = None
    if sbr_writers is not None:
        states = (C.c_void_p * len(ids))(*[w.buf.ctypes.data if w is not None else None for w in sbr_writers])
    buf = np.zeros(1 << 17, np.uint8)
    out = []
    for f in range(batch.n_frames):
        cf = f * nch
        q = np.ascontiguousarray(batch.q[cf:cf + nch])
        sf = np.ascontiguousarray(batch.sf[cf:cf + nch])
        cb = np.ascontiguousarray(batch.cb[cf:cf + nch])
        ics = np.ascontiguousarray(batch.ics[cf:cf + nch])
        ms = np.ascontiguousarray(batch.ms_used[f]) if batch.ms_used is not None else np.zeros(16, np.uint64)
        lst = cces[f] if f < len(cces) else []
        n = len(lst)
        d = np.zeros(max(n, 1), CCE_DESC_DTYPE)
        cq = np.zeros((max(n, 1), 1024), np.int16)
        csf = np.zeros((max(n, 1), 128), np.uint8)
        ccb = np.zeros((max(n, 1), 128), np.uint8)
        import jaadec_amd.native as N
        cics = np.zeros(max(n, 1), N.ICS_DTYPE)
        for k, (dk, qk, sfk, cbk, icsk) in enumerate(lst):
            d[k], cq[k], csf[k], ccb[k], cics[k] = dk, qk, sfk, cbk, icsk
        rec = np.ascontiguousarray(batch.sbr[f]).reshape(-1) if states is not None else None
        r = lib().jaad_write_frame_cce_sbr(sf_index, len(ids), ids_a, q.ctypes.data, sf.ctypes.data, cb.ctypes.data,
                                           ics.ctypes.data, ms.ctypes.data, n, d.ctypes.data, cq.ctypes.data,
                                           csf.ctypes.data, ccb.ctypes.data, cics.ctypes.data,
                                           rec.ctypes.data if rec is not None else None, states, buf.ctypes.data,
                                           buf.nbytes)
        if r < 0:
            raise ValueError(f"frame {f} cannot be written")
        out.append(buf[:r].tobytes())
    return out


def decode_batch_mc(sf_index: int, batch, ids, flags: int = 0, threads: int = 1, tns_mode: int = 0,
                    sbr: bool = False, down: bool = False) -> np.ndarray:
    """TEST ORACLE for a multichannel batch, from fresh stream states: every element decoded on its
    own (SCE/LFE as a mono, CPE as a stereo stream: SyntacticElements.process runs them in turn)
    and the channels interleaved in element order (SampleBuffer.accept); uint8 [n_frames, bytes].
    With sbr (multichannel HE-AAC, batch.sbr [frame][element]): each element runs its own SBR
    (SCE: SBR1, whose dataL and dataR are both output, A/syntax/SCE.java:115-132; CPE: SBR2,
    A/syntax/CPE.java:195-204); the LFE has no SBR data and is upsampled (one channel)."""
    import jaadec_amd.native as N

    nf, nch = batch.n_frames, batch.nch
    fb = 4 if flags & 2 else 2
    planes = []
    c, cpe = 0, 0
    for e_idx, i in enumerate(ids):
        k = 2 if i == 1 else 1
        cfr = (np.arange(nf)[:, None] * nch + c + np.arange(k)[None, :]).reshape(-1)
        el = N.Batch(np.ascontiguousarray(batch.q[cfr]), np.ascontiguousarray(batch.sf[cfr]),
                     np.ascontiguousarray(batch.cb[cfr]), np.ascontiguousarray(batch.ics[cfr]),
                     np.ascontiguousarray(batch.ms_used[:, 2 * cpe:2 * cpe + 2]) if k == 2 else None,
                     np.ascontiguousarray(batch.tns[cfr]) if batch.tns is not None else None,
                     batch.stream_slot.copy(), batch.frame_begin.copy(), k)
        el.frame_status = batch.frame_status
        if batch.cce_terms is not None:  # the element's coupling terms, channels relative to it
            t = batch.cce_terms[(batch.cce_terms["channel"] >= c) & (batch.cce_terms["channel"] < c + k)].copy()
            t["channel"] -= c
            el.cce_q, el.cce_sf, el.cce_cb, el.cce_ics = batch.cce_q, batch.cce_sf, batch.cce_cb, batch.cce_ics
            el.cce_terms = np.ascontiguousarray(t)
        cfg = N.make_cfg(sf_index, 2 if k == 2 else 1, tns_mode, sbr=sbr, down=down)
        if sbr:
            el.sbr = np.ascontiguousarray(batch.sbr[:, e_idx])
        pcm = decode_batch(cfg, el, Streams(int(batch.stream_slot.max()) + 1), flags, threads)
        dt = np.uint32 if fb == 4 else np.uint16
        frames = pcm.view(dt).reshape(nf, -1, 2)
        out_ch = (1 if i == 3 else 2) if sbr else k
        planes += [frames[:, :, j] for j in range(out_ch)]
        c += k
        cpe += k == 2
    return np.ascontiguousarray(np.stack(planes, 2)).view(np.uint8).reshape(nf, -1)


def adts_wrap(payloads: list, sf_index: int, channel_config: int) -> bytes:
    """TEST WRITER: an ADTS stream (no CRC) of raw_data_block payloads."""
    hdr = np.zeros(7, np.uint8)
    parts = []
    for p in payloads:
        lib().jaad_write_adts_header(sf_index, channel_config, len(p), hdr.ctypes.data)
        parts += [hdr.tobytes(), p]
    return b"".join(parts)


class Streams:
    """Per-slot restated decoder state (orc_stream: ICStream.overlap per channel + SBR object)."""

    def __init__(self, n_slots: int):
        self.n = n_slots
        self.state = np.zeros((n_slots, lib().orc_stream_bytes()), np.uint8)

    def __del__(self):
        if _lib is not None and getattr(self, "state", None) is not None:
            _lib.orc_streams_free(self.state.ctypes.data, self.n)


def decode_batch(cfg, batch, streams: Streams, flags: int = 0, threads: int = 1) -> np.ndarray:
    """Decode a jaadec_amd.native.Batch on the CPU restatement; returns uint8 [n_frames, bytes]."""
    down = cfg.sbr and cfg.ext_sf_index == cfg.sf_index  # downsampled SBR: core-rate output
    nb = (2048 if cfg.sbr and not down else 1024) * 2 * (4 if flags & 2 else 2)
    drops = getattr(batch, "frame_status", None) is not None and bool(np.any(batch.frame_status))
    out = (np.zeros if drops else np.empty)((batch.n_frames, nb), np.uint8)  # dropped frames: rows stay 0
    bs = batch.struct()
    if threads == 1:
        rc = lib().orc_decode_batch(C.addressof(cfg), streams.state.ctypes.data, C.addressof(bs), out.ctypes.data,
                                    out.nbytes, flags)
    else:
        rc = lib().orc_decode_batch_mt(C.addressof(cfg), streams.state.ctypes.data, C.addressof(bs),
                                       out.ctypes.data, out.nbytes, flags, threads)
    if rc:
        raise RuntimeError(f"oracle decode failed: {rc}")
    return out
