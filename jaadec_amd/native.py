"""ctypes binding of the C-ABI (include/jaad_gpu.h, include/jaad_synth.h).

The product path is ``libjaadgpu.so`` (HIP kernels for gfx950).  There is deliberately no CPU
fallback: if the library cannot be loaded, or no gfx950 device is present when a context is
created, the call raises.
"""
from __future__ import annotations

import ctypes as C
from dataclasses import dataclass
from pathlib import Path

import numpy as np

PKG = Path(__file__).resolve().parent
import os as _os
LIB_PATH = Path(_os.environ["JAAD_LIB"]) if _os.environ.get("JAAD_LIB") else PKG / "libjaadgpu.so"
SYNTH_PATH = PKG / "libjaadsynth.so"

ABI_VERSION = 4

# status codes (jaad_status)
OK, ERR_INVALID_ARG, ERR_NO_DEVICE, ERR_HIP, ERR_UNSUPPORTED, ERR_BITSTREAM, ERR_NOMEM, ERR_ABI, ERR_EOS = 0, -1, -2, -3, -4, -5, -6, -7, -8
CCE_MAX_RECORDS = 65536  # jaad_gpu.h JAAD_CCE_MAX_RECORDS (16-bit jaad_cce_term.cce)
CCE_GAIN_MAX = float(2 ** 60)  # jaad_gpu.h JAAD_CCE_GAIN_MAX

ONLY_LONG_SEQUENCE, LONG_START_SEQUENCE, EIGHT_SHORT_SEQUENCE, LONG_STOP_SEQUENCE = 0, 1, 2, 3
ZERO_HCB, NOISE_HCB, INTENSITY_HCB2, INTENSITY_HCB = 0, 13, 14, 15
TNS_COMPAT, TNS_SPEC = 0, 1
PRECISION_EXACT, PRECISION_LSB1 = 0, 1  # jaad_stream_cfg.precision (JAAD_PRECISION_*)
PCM_BIG_ENDIAN, PCM_LITTLE_ENDIAN, PCM_FLOAT32 = 0, 1, 2
HINT_SHORT_WINDOWS = 1 << 8  # jaad_decode_batch_device: the batch holds EIGHT_SHORT frames (kernel choice only)
ICS_HAS_PNS, ICS_HAS_IS, ICS_TNS, ICS_MS_PRESENT, ICS_COMMON_WINDOW = 1, 2, 4, 8, 16

ICS_DTYPE = np.dtype([
    ("window_sequence", "u1"), ("window_shape", "u1"), ("window_shape_prev", "u1"), ("max_sfb", "u1"),
    ("grouping", "u1"), ("flags", "u1"), ("reserved", "u1", (2,)), ("pns_state", "<u4"), ("reserved2", "<u4"),
])
assert ICS_DTYPE.itemsize == 16
TNS_FILTER_DTYPE = np.dtype([("window", "u1"), ("length", "u1"), ("order", "u1"), ("flags", "u1"), ("coef", "u1", (20,))])
TNS_DTYPE = np.dtype([("n_filters", "u1"), ("reserved", "u1", (3,)), ("filt", TNS_FILTER_DTYPE, (8,))])
assert TNS_DTYPE.itemsize == 196

SBR_HEADER_DTYPE = np.dtype([(n, "u1") for n in (
    "amp_res", "start_freq", "stop_freq", "xover_band", "freq_scale", "alter_scale", "noise_bands",
    "limiter_bands", "limiter_gains", "interpol_freq", "smoothing_mode", "reserved")])
SBR_CHANNEL_DTYPE = np.dtype([
    ("add_harmonic", "<u8"), ("E", "<i2", (5, 64)), ("Q", "<i2", (2, 8)), ("frame_class", "u1"), ("L_E", "u1"),
    ("L_Q", "u1"), ("bs_pointer", "u1"), ("t_E", "u1", (6,)), ("t_Q", "u1", (3,)), ("f", "u1", (6,)),
    ("invf_mode", "u1", (5,)), ("add_harmonic_flag", "u1"), ("reserved", "u1", (7,))])
PS_FRAME_DTYPE = np.dtype([("iid_mode", "u1"), ("icc_mode", "u1"), ("num_env", "u1"), ("nr_ipdopd_par", "u1"),
                           ("border", "u1", (6,)), ("reserved", "u1", (2,)), ("iid", "i1", (5, 34)),
                           ("icc", "i1", (5, 34)), ("ipd", "i1", (5, 17)), ("opd", "i1", (5, 17)),
                           ("pad", "u1", (6,))])
SBR_OK, SBR_UPSAMPLE = 0, 1  # jaad_sbr_frame.status
SBR_FRAME_DTYPE = np.dtype([("header_present", "u1"), ("coupling", "u1"), ("ps_present", "u1"), ("status", "u1"),
                            ("hdr", SBR_HEADER_DTYPE), ("ch", SBR_CHANNEL_DTYPE, (2,)), ("ps", PS_FRAME_DTYPE)])
assert SBR_CHANNEL_DTYPE.itemsize == 712 and PS_FRAME_DTYPE.itemsize == 528 and SBR_FRAME_DTYPE.itemsize == 1968
# jaad_cce_term (include/jaad_gpu.h): one dependent-coupling application
CCE_TERM_DTYPE = np.dtype([("frame", "<u4"), ("channel", "u1"), ("point", "u1"), ("cce", "<u2"), ("gain", "<f4", (120,))])
assert CCE_TERM_DTYPE.itemsize == 488


class StreamCfg(C.Structure):
    _fields_ = [("abi_version", C.c_uint32), ("profile", C.c_uint8), ("sf_index", C.c_uint8),
                ("channel_config", C.c_uint8), ("tns_mode", C.c_uint8), ("sbr", C.c_uint8), ("ps", C.c_uint8),
                ("ext_sf_index", C.c_uint8), ("precision", C.c_uint8)]


class BatchStruct(C.Structure):
    _fields_ = [("n_frames", C.c_uint32), ("n_runs", C.c_uint32), ("stream_slot", C.c_void_p),
                ("frame_begin", C.c_void_p), ("q", C.c_void_p), ("sf", C.c_void_p), ("cb", C.c_void_p),
                ("ics", C.c_void_p), ("ms_used", C.c_void_p), ("tns", C.c_void_p), ("sbr", C.c_void_p),
                ("n_cce", C.c_uint32), ("n_cce_terms", C.c_uint32), ("cce_q", C.c_void_p), ("cce_sf", C.c_void_p),
                ("cce_cb", C.c_void_p), ("cce_ics", C.c_void_p), ("cce_terms", C.c_void_p),
                ("frame_status", C.c_void_p)]

# jaad_batch.frame_status values (JAAD_FRAME_*)
FRAME_DECODE, FRAME_EOS = 0, 1


class SynthParams(C.Structure):
    _fields_ = [("seed", C.c_uint64), ("n_streams", C.c_uint32), ("frames_per_stream", C.c_uint32),
                ("sf_index", C.c_uint8), ("channel_config", C.c_uint8), ("window_switching", C.c_uint8),
                ("tns_percent", C.c_uint8), ("pns_percent", C.c_uint8), ("is_percent", C.c_uint8),
                ("ms_mode", C.c_uint8), ("global_gain", C.c_uint8), ("escape_permille", C.c_uint8),
                ("common_window", C.c_uint8), ("sbr", C.c_uint8), ("sbr_level", C.c_uint8),
                ("pns_state0", C.c_uint32), ("coupling_percent", C.c_uint8), ("upsample_percent", C.c_uint8),
                ("nohdr_frames", C.c_uint8), ("reserved", C.c_uint8), ("first_stream", C.c_uint32)]


# every symbol include/jaad_gpu.h declares (checked by tests/test_abi.py)
EXPORTS = ["jaad_cfg_sample_length", "jaad_cfg_channel_count", "jaad_frame_pcm_bytes", "jaad_ctx_create",
           "jaad_ctx_destroy", "jaad_ctx_core_channels", "jaad_decode_batch", "jaad_decode_batch_device", "jaad_wait", "jaad_state_bytes",
           "jaad_state_export", "jaad_state_import", "jaad_state_reset", "jaad_strerror", "jaad_last_error",
           "jaad_host_register", "jaad_host_unregister", "jaad_host_alloc", "jaad_host_free"]
# every symbol include/jaad_parse.h declares
PARSE_EXPORTS = ["jaad_asc_parse", "jaad_adts_find", "jaad_adts_cfg", "jaad_raw_pce_cfg", "jaad_parser_create", "jaad_parser_destroy",
                 "jaad_parser_clone", "jaad_parser_copy",
                 "jaad_parser_pns_state", "jaad_parser_set_pns_state", "jaad_parse_frame", "jaad_probe_sbr"]


class AdtsHeader(C.Structure):
    _fields_ = [("profile", C.c_uint8), ("sf_index", C.c_uint8), ("channel_config", C.c_uint8),
                ("protection_absent", C.c_uint8), ("n_raw_blocks", C.c_uint8), ("reserved", C.c_uint8 * 3),
                ("frame_length", C.c_uint32), ("header_bytes", C.c_uint32)]


class FrameOut(C.Structure):
    _fields_ = [("q", C.c_void_p), ("sf", C.c_void_p), ("cb", C.c_void_p), ("ics", C.c_void_p),
                ("ms_used", C.c_void_p), ("tns", C.c_void_p), ("sbr", C.c_void_p),
                ("cce_q", C.c_void_p), ("cce_sf", C.c_void_p), ("cce_cb", C.c_void_p), ("cce_ics", C.c_void_p),
                ("cce_terms", C.c_void_p), ("cce_cap", C.c_uint32), ("term_cap", C.c_uint32),
                ("n_cce", C.c_uint32), ("n_cce_terms", C.c_uint32)]


class JaadError(RuntimeError):
    """Raised for a nonzero jaad_status (the JNI glue maps these to AACException)."""

    def __init__(self, status: int, what: str = ""):
        self.status = status
        super().__init__(f"{what}: {status} ({strerror(status)})" if what else f"{status} ({strerror(status)})")


_lib = None
_synth = None


def lib() -> C.CDLL:
    global _lib
    if _lib is None:
        if not LIB_PATH.exists():
            raise RuntimeError(f"{LIB_PATH} is missing: build it with `python -m jaadec_amd.build` "
                               "(there is no CPU fallback for the HIP path)")
        _lib = load_lib(LIB_PATH)
    return _lib


def load_lib(path) -> C.CDLL:
    """The C-ABI of one libjaadgpu.so build with its prototypes (lib() holds the product's; A/B
    timing scripts load variants side by side)."""
    L = C.CDLL(str(path))
    L.jaad_cfg_sample_length.argtypes = [C.POINTER(StreamCfg)]
    L.jaad_cfg_channel_count.argtypes = [C.POINTER(StreamCfg)]
    L.jaad_frame_pcm_bytes.argtypes = [C.POINTER(StreamCfg), C.c_uint32]
    L.jaad_frame_pcm_bytes.restype = C.c_size_t
    L.jaad_ctx_create.argtypes = [C.POINTER(StreamCfg), C.c_uint32, C.c_int, C.POINTER(C.c_void_p)]
    L.jaad_ctx_destroy.argtypes = [C.c_void_p]
    L.jaad_ctx_destroy.restype = None
    L.jaad_ctx_core_channels.argtypes = [C.c_void_p]
    L.jaad_decode_batch.argtypes = [C.c_void_p, C.POINTER(BatchStruct), C.c_void_p, C.c_size_t, C.c_uint32]
    L.jaad_decode_batch_device.argtypes = [C.c_void_p, C.POINTER(BatchStruct), C.c_void_p, C.c_size_t,
                                           C.c_uint32, C.c_void_p]
    L.jaad_wait.argtypes = [C.c_void_p]
    L.jaad_host_register.argtypes = [C.c_void_p, C.c_void_p, C.c_size_t]
    L.jaad_host_unregister.argtypes = [C.c_void_p, C.c_void_p]
    L.jaad_host_alloc.argtypes = [C.c_void_p, C.c_size_t, C.POINTER(C.c_void_p)]
    L.jaad_host_free.argtypes = [C.c_void_p, C.c_void_p]
    L.jaad_state_bytes.argtypes = [C.c_void_p]
    L.jaad_state_bytes.restype = C.c_size_t
    L.jaad_state_export.argtypes = [C.c_void_p, C.c_uint32, C.c_void_p, C.c_size_t]
    L.jaad_state_import.argtypes = [C.c_void_p, C.c_uint32, C.c_void_p, C.c_size_t]
    L.jaad_state_reset.argtypes = [C.c_void_p, C.c_uint32]
    L.jaad_strerror.argtypes = [C.c_int]
    L.jaad_strerror.restype = C.c_char_p
    L.jaad_last_error.argtypes = [C.c_void_p]
    L.jaad_last_error.restype = C.c_char_p
    L.jaad_asc_parse.argtypes = [C.c_char_p, C.c_size_t, C.POINTER(StreamCfg)]
    L.jaad_adts_find.argtypes = [C.c_void_p, C.c_size_t, C.POINTER(C.c_size_t), C.POINTER(AdtsHeader)]
    L.jaad_adts_cfg.argtypes = [C.POINTER(AdtsHeader), C.POINTER(StreamCfg)]
    L.jaad_raw_pce_cfg.argtypes = [C.c_char_p, C.c_size_t, C.POINTER(StreamCfg)]
    L.jaad_parser_create.argtypes = [C.POINTER(StreamCfg), C.POINTER(C.c_void_p)]
    L.jaad_parser_destroy.argtypes = [C.c_void_p]
    L.jaad_parser_clone.argtypes = [C.c_void_p, C.POINTER(C.c_void_p)]
    L.jaad_parser_copy.argtypes = [C.c_void_p, C.c_void_p]
    L.jaad_parser_destroy.restype = None
    L.jaad_parser_pns_state.argtypes = [C.c_void_p]
    L.jaad_parser_pns_state.restype = C.c_uint32
    L.jaad_parser_set_pns_state.argtypes = [C.c_void_p, C.c_uint32]
    L.jaad_parser_set_pns_state.restype = None
    L.jaad_parse_frame.argtypes = [C.c_void_p, C.c_char_p, C.c_size_t, C.POINTER(FrameOut)]
    L.jaad_probe_sbr.argtypes = [C.POINTER(StreamCfg), C.c_char_p, C.c_size_t, C.POINTER(C.c_uint32)]
    return L


def synth_lib() -> C.CDLL:
    global _synth
    if _synth is None:
        if not SYNTH_PATH.exists():
            raise RuntimeError(f"{SYNTH_PATH} is missing: build with `python -m jaadec_amd.build`")
        S = C.CDLL(str(SYNTH_PATH))
        S.jaad_synth_default.argtypes = [C.c_int, C.POINTER(SynthParams)]
        S.jaad_synth_default.restype = None
        S.jaad_synth_generate.argtypes = [C.POINTER(SynthParams)] + [C.c_void_p] * 8 + [C.c_int]
        S.jaad_synth_sbr.argtypes = [C.POINTER(SynthParams), C.c_void_p, C.c_int]
        _synth = S
    return _synth


def strerror(status: int) -> str:
    try:
        return lib().jaad_strerror(status).decode()
    except Exception:  # pragma: no cover - library missing
        return "?"


def _ptr(a):
    return None if a is None else a.ctypes.data


@dataclass
class Batch:
    """Host SoA batch in the jaad_gpu.h layout (numpy arrays)."""

    q: np.ndarray            # int16 [ncf, 1024]
    sf: np.ndarray           # uint8 [ncf, 128]
    cb: np.ndarray           # uint8 [ncf, 128]
    ics: np.ndarray          # ICS_DTYPE [ncf]
    ms_used: np.ndarray | None  # uint64 [nf, 2]
    tns: np.ndarray | None      # TNS_DTYPE [ncf]
    stream_slot: np.ndarray  # uint32 [n_runs]
    frame_begin: np.ndarray  # uint32 [n_runs+1]
    nch: int
    sbr: np.ndarray | None = None  # SBR_FRAME_DTYPE [nf] (host) when the config has SBR
    # dependent coupling (jaad_cce_term): CCE records and the terms applying them (None: no CCEs)
    cce_q: np.ndarray | None = None     # int16 [n_cce, 1024]
    cce_sf: np.ndarray | None = None    # uint8 [n_cce, 128]
    cce_cb: np.ndarray | None = None    # uint8 [n_cce, 128]
    cce_ics: np.ndarray | None = None   # ICS_DTYPE [n_cce]
    cce_terms: np.ndarray | None = None  # CCE_TERM_DTYPE [n_terms], sorted by frame
    # per-frame status (uint8 [nf] of FRAME_*; None: every frame decodes): FRAME_EOS frames are
    # dropped as Decoder.decodeFrame drops them (A/Decoder.java:89-101), PCM slot untouched
    frame_status: np.ndarray | None = None

    @property
    def n_frames(self) -> int:
        return int(self.frame_begin[-1])

    @property
    def n_cce(self) -> int:
        return 0 if self.cce_ics is None else len(self.cce_ics)

    def struct(self) -> BatchStruct:
        for a in (self.q, self.sf, self.cb, self.ics, self.stream_slot, self.frame_begin):
            assert a.flags["C_CONTIGUOUS"]
        nt = 0 if self.cce_terms is None else len(self.cce_terms)
        return BatchStruct(self.n_frames, len(self.stream_slot), _ptr(self.stream_slot), _ptr(self.frame_begin),
                           _ptr(self.q), _ptr(self.sf), _ptr(self.cb), _ptr(self.ics), _ptr(self.ms_used),
                           _ptr(self.tns), _ptr(self.sbr), self.n_cce, nt, _ptr(self.cce_q), _ptr(self.cce_sf),
                           _ptr(self.cce_cb), _ptr(self.cce_ics), _ptr(self.cce_terms), _ptr(self._status()))

    def _status(self) -> np.ndarray | None:
        if self.frame_status is None:
            return None
        st = np.ascontiguousarray(self.frame_status, np.uint8)
        if st.shape != (self.n_frames,):
            raise ValueError("frame_status: one uint8 per frame expected")
        self.frame_status = st
        return st

    def _cce_for(self, frames: np.ndarray) -> dict:
        """The coupling of the given (renumbered in order) frames: all CCE records kept, the terms
        of those frames with their frame indices renumbered."""
        if self.cce_terms is None:
            return {}
        pos = np.full(self.n_frames, -1, np.int64)
        pos[frames] = np.arange(len(frames))
        t = self.cce_terms[pos[self.cce_terms["frame"]] >= 0].copy()
        t["frame"] = pos[t["frame"]]
        t = t[np.argsort(t["frame"], kind="stable")]
        return dict(cce_q=self.cce_q, cce_sf=self.cce_sf, cce_cb=self.cce_cb, cce_ics=self.cce_ics,
                    cce_terms=np.ascontiguousarray(t))

    def select_runs(self, runs) -> "Batch":
        """Sub-batch made of the given runs (frames renumbered, slots kept)."""
        runs = list(runs)
        fb = self.frame_begin
        frames = np.concatenate([np.arange(fb[r], fb[r + 1]) for r in runs]) if runs else np.zeros(0, np.int64)
        cfr = (frames[:, None] * self.nch + np.arange(self.nch)[None, :]).reshape(-1)
        lens = np.array([fb[r + 1] - fb[r] for r in runs], np.uint32)
        begin = np.zeros(len(runs) + 1, np.uint32)
        begin[1:] = np.cumsum(lens)
        return Batch(np.ascontiguousarray(self.q[cfr]), np.ascontiguousarray(self.sf[cfr]),
                     np.ascontiguousarray(self.cb[cfr]), np.ascontiguousarray(self.ics[cfr]),
                     None if self.ms_used is None else np.ascontiguousarray(self.ms_used[frames]),
                     None if self.tns is None else np.ascontiguousarray(self.tns[cfr]),
                     np.ascontiguousarray(self.stream_slot[runs]).astype(np.uint32), begin, self.nch,
                     None if self.sbr is None else np.ascontiguousarray(self.sbr[frames]), **self._cce_for(frames),
                     frame_status=None if self.frame_status is None else np.ascontiguousarray(self.frame_status[frames]))

    def split_frames(self, cut: int) -> tuple["Batch", "Batch"]:
        """Split every run at its frame `cut` (for multi-call continuation tests)."""
        fb = self.frame_begin
        a_frames, b_frames, la, lb = [], [], [], []
        for r in range(len(self.stream_slot)):
            f0, f1 = int(fb[r]), int(fb[r + 1])
            m = min(f0 + cut, f1)
            a_frames.append(np.arange(f0, m))
            b_frames.append(np.arange(m, f1))
            la.append(m - f0)
            lb.append(f1 - m)

        def mk(fr, lens):
            frames = np.concatenate(fr)
            cfr = (frames[:, None] * self.nch + np.arange(self.nch)[None, :]).reshape(-1)
            begin = np.zeros(len(lens) + 1, np.uint32)
            begin[1:] = np.cumsum(lens)
            return Batch(np.ascontiguousarray(self.q[cfr]), np.ascontiguousarray(self.sf[cfr]),
                         np.ascontiguousarray(self.cb[cfr]), np.ascontiguousarray(self.ics[cfr]),
                         None if self.ms_used is None else np.ascontiguousarray(self.ms_used[frames]),
                         None if self.tns is None else np.ascontiguousarray(self.tns[cfr]),
                         self.stream_slot.copy(), begin, self.nch,
                         None if self.sbr is None else np.ascontiguousarray(self.sbr[frames]), **self._cce_for(frames),
                         frame_status=None if self.frame_status is None else np.ascontiguousarray(self.frame_status[frames]))

        return mk(a_frames, la), mk(b_frames, lb)


def synth_params(config_id: int = 2, **over) -> SynthParams:
    p = SynthParams()
    synth_lib().jaad_synth_default(config_id, C.byref(p))
    for k, v in over.items():
        setattr(p, k, v)
    return p


def synth_batch(p: SynthParams, with_tns: bool | None = None, threads: int = 0) -> Batch:
    nch = 2 if p.channel_config == 2 else 1
    nf = p.n_streams * p.frames_per_stream
    ncf = nf * nch
    q = np.empty((ncf, 1024), np.int16)
    sf = np.empty((ncf, 128), np.uint8)
    cb = np.empty((ncf, 128), np.uint8)
    ics = np.empty(ncf, ICS_DTYPE)
    ms = np.zeros((nf, 2), np.uint64) if nch == 2 else None
    if with_tns is None:
        with_tns = p.tns_percent > 0
    tns = np.zeros(ncf, TNS_DTYPE) if with_tns else None
    slot = np.empty(p.n_streams, np.uint32)
    begin = np.empty(p.n_streams + 1, np.uint32)
    rc = synth_lib().jaad_synth_generate(C.byref(p), _ptr(q), _ptr(sf), _ptr(cb), _ptr(ics), _ptr(ms), _ptr(tns),
                                         _ptr(slot), _ptr(begin), threads)
    if rc:
        raise JaadError(rc, "jaad_synth_generate")
    sbr = None
    if p.sbr:
        sbr = np.zeros(nf, SBR_FRAME_DTYPE)
        rc = synth_lib().jaad_synth_sbr(C.byref(p), _ptr(sbr), threads)
        if rc:
            raise JaadError(rc, "jaad_synth_sbr")
    return Batch(q, sf, cb, ics, ms, tns, slot, begin, nch, sbr)


def make_cfg(sf_index: int = 3, channel_config: int = 2, tns_mode: int = TNS_COMPAT, sbr: bool = False,
             ps: bool = False, down: bool = False, precision: int = PRECISION_EXACT) -> StreamCfg:
    """jaad_stream_cfg; with sbr the output rate is twice the core rate (index - 3), or the core
    rate itself with down (downsampled SBR: extension rate = core rate).  precision:
    PRECISION_EXACT (bit-identical to the reference's arithmetic) or PRECISION_LSB1 (+-1 LSB)."""
    sbr = sbr or ps
    return StreamCfg(ABI_VERSION, 2, sf_index, channel_config, tns_mode, int(sbr), int(ps),
                     (sf_index if down else sf_index - 3) if sbr else 0, precision)


def sbr_downsampled(cfg: StreamCfg) -> bool:
    return bool(cfg.sbr) and cfg.ext_sf_index == cfg.sf_index


def cfg_for(p: SynthParams, tns_mode: int = TNS_COMPAT, precision: int = PRECISION_EXACT) -> StreamCfg:
    return make_cfg(p.sf_index, p.channel_config, tns_mode, bool(p.sbr), p.sbr == 2, precision=precision)


# channel elements of the AAC-LC multichannel configurations (0 SCE, 1 CPE, 3 LFE; ISO/IEC 14496-3
# Table 1.19), in bitstream order
MC_ELEMENTS = {3: (0, 1), 4: (0, 1, 0), 5: (0, 1, 1), 6: (0, 1, 1, 3), 7: (0, 1, 1, 1, 3)}


def core_channels(cfg) -> int:
    """Channel-frame records per frame of a configuration (jaad_ctx_core_channels)."""
    cc = cfg.channel_config
    if cc in MC_ELEMENTS:
        return sum(2 if e == 1 else 1 for e in MC_ELEMENTS[cc])
    return 2 if cc == 2 else 1


def n_cpe(cfg) -> int:
    cc = cfg.channel_config
    return sum(e == 1 for e in MC_ELEMENTS[cc]) if cc in MC_ELEMENTS else int(cc == 2)


def n_elements(cfg) -> int:
    """Channel elements per frame (one jaad_sbr_frame each in a multichannel HE-AAC batch)."""
    cc = cfg.channel_config
    return len(MC_ELEMENTS[cc]) if cc in MC_ELEMENTS else 1


def out_channels(cfg) -> int:
    """PCM channels per sample instant (jaad_cfg_channel_count): 2 for mono/stereo (an SCE's output is
    duplicated); multichannel AAC-LC: the core channels; multichannel HE-AAC: every SCE and CPE gives
    two (SCE.process with SBR accepts dataL and dataR, A/syntax/SCE.java:122-129), an LFE one."""
    cc = cfg.channel_config
    if cc not in MC_ELEMENTS:
        return 2
    if not cfg.sbr:
        return core_channels(cfg)
    return sum(1 if e == 3 else 2 for e in MC_ELEMENTS[cc])


def mc_batch(elements: list, ids) -> "Batch":
    """One multichannel batch (all channels' records per frame, element order) from per-element
    batches of the same runs (SCE/LFE: 1 channel, CPE: 2 with ms_used)."""
    nf = elements[0].n_frames
    nch = sum(e.nch for e in elements)
    cols = lambda name, w: np.concatenate([getattr(e, name).reshape(nf, e.nch, *w) for e in elements], 1)
    q = np.ascontiguousarray(cols("q", (1024,)).reshape(nf * nch, 1024))
    sf = np.ascontiguousarray(cols("sf", (128,)).reshape(nf * nch, 128))
    cb = np.ascontiguousarray(cols("cb", (128,)).reshape(nf * nch, 128))
    ics = np.ascontiguousarray(cols("ics", ()).reshape(nf * nch))
    cpes = [e for e, i in zip(elements, ids) if i == 1]
    ms = np.ascontiguousarray(np.concatenate([e.ms_used for e in cpes], 1)) if cpes else None
    tns = None
    if any(e.tns is not None for e in elements):
        tns = np.zeros((nf, nch), TNS_DTYPE)
        c = 0
        for e in elements:
            if e.tns is not None:
                tns[:, c:c + e.nch] = e.tns.reshape(nf, e.nch)
            c += e.nch
        tns = tns.reshape(nf * nch)
    sbr = None
    if any(e.sbr is not None for e in elements):
        # multichannel HE-AAC: one record per element per frame; an element without records (the
        # LFE) is upsampled (JAAD_SBR_UPSAMPLE)
        sbr = np.zeros((nf, len(elements)), SBR_FRAME_DTYPE)
        for k, e in enumerate(elements):
            if e.sbr is not None:
                sbr[:, k] = e.sbr
            else:
                sbr[:, k]["status"] = SBR_UPSAMPLE
    return Batch(q, sf, cb, ics, ms, tns, elements[0].stream_slot.copy(), elements[0].frame_begin.copy(), nch, sbr)


def pcm_frame_bytes(flags: int, sbr: bool = False, down: bool = False) -> int:
    return (2048 if sbr and not down else 1024) * 2 * (4 if flags & PCM_FLOAT32 else 2)


class Context:
    """Owns a jaad_ctx: n_slots independent stream states on one gfx950 device."""

    def __init__(self, cfg: StreamCfg, n_slots: int, device: int = 0):
        self.cfg = cfg
        self.n_slots = n_slots
        h = C.c_void_p()
        rc = lib().jaad_ctx_create(C.byref(cfg), n_slots, device, C.byref(h))
        if rc:
            raise JaadError(rc, "jaad_ctx_create")
        self.h = h

    def close(self):
        h = getattr(self, "h", None)
        if h:
            self.h = None
            lib().jaad_ctx_destroy(h)

    def __del__(self):
        try:
            self.close()
        except TypeError:  # interpreter shutdown: this module's globals (lib) are already gone
            pass

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.close()

    def _check(self, rc: int, what: str):
        if rc:
            detail = lib().jaad_last_error(self.h).decode()
            raise JaadError(rc, f"{what} {detail}".strip())

    def decode(self, batch: Batch, flags: int = PCM_BIG_ENDIAN, out: np.ndarray | None = None) -> np.ndarray:
        """Host-buffer batch decode -> PCM bytes (uint8 [n_frames, frame_bytes]), into `out` when
        given (e.g. a buffer registered with register()).  The rows of dropped frames
        (batch.frame_status) are left as they are: zero in a fresh output."""
        nb = lib().jaad_frame_pcm_bytes(C.byref(self.cfg), flags)
        if out is None:
            drops = batch.frame_status is not None and bool(np.any(batch.frame_status))
            out = (np.zeros if drops else np.empty)((batch.n_frames, nb), np.uint8)
        assert out.flags["C_CONTIGUOUS"] and out.nbytes >= batch.n_frames * nb
        bs = batch.struct()
        self._check(lib().jaad_decode_batch(self.h, C.byref(bs), _ptr(out), out.nbytes, flags), "jaad_decode_batch")
        return out

    def wait(self) -> None:
        """Wait for every call queued on the context (jaad_wait)."""
        self._check(lib().jaad_wait(self.h), "jaad_wait")

    def register(self, *arrays: np.ndarray) -> None:
        """Page-lock host arrays reused across decode() calls (jaad_host_register)."""
        for a in arrays:
            if a is not None and a.nbytes:
                self._check(lib().jaad_host_register(self.h, _ptr(a), a.nbytes), "jaad_host_register")

    def unregister(self, *arrays: np.ndarray) -> None:
        for a in arrays:
            if a is not None and a.nbytes:
                self._check(lib().jaad_host_unregister(self.h, _ptr(a)), "jaad_host_unregister")

    def host_array(self, shape, dtype=np.uint8) -> np.ndarray:
        """A numpy array in page-locked memory owned by the context (jaad_host_alloc): batch arrays
        and PCM buffers placed in it are copied by DMA directly.  Valid until free_host() or close()."""
        dt = np.dtype(dtype)
        n = max(int(np.prod(shape)) * dt.itemsize, 1)
        p = C.c_void_p()
        self._check(lib().jaad_host_alloc(self.h, n, C.byref(p)), "jaad_host_alloc")
        buf = (C.c_uint8 * n).from_address(p.value)
        return np.frombuffer(buf, np.uint8, int(np.prod(shape)) * dt.itemsize).view(dt).reshape(shape)

    def free_host(self, *arrays: np.ndarray) -> None:
        for a in arrays:
            if a is not None:
                self._check(lib().jaad_host_free(self.h, _ptr(a)), "jaad_host_free")

    def host_batch(self, b: "Batch") -> "Batch":
        """A copy of b whose arrays live in host_array() memory (free with free_host(*arrays))."""
        def cp(a):
            if a is None:
                return None
            h = self.host_array(a.shape, a.dtype)
            h[...] = a
            return h
        return Batch(cp(b.q), cp(b.sf), cp(b.cb), cp(b.ics), cp(b.ms_used), cp(b.tns), b.stream_slot, b.frame_begin,
                     b.nch, b.sbr, b.cce_q, b.cce_sf, b.cce_cb, b.cce_ics, b.cce_terms)

    def decode_device(self, dev: dict, batch: Batch, pcm_dev_ptr: int, pcm_bytes: int, flags: int = 0,
                      stream_ptr: int | None = None) -> None:
        """Device-resident decode: dev maps array names to device pointers (ints)."""
        nt = 0 if batch.cce_terms is None else len(batch.cce_terms)
        bs = BatchStruct(batch.n_frames, len(batch.stream_slot), _ptr(batch.stream_slot), _ptr(batch.frame_begin),
                         dev["q"], dev["sf"], dev["cb"], dev["ics"], dev.get("ms_used"), dev.get("tns"),
                         _ptr(batch.sbr), batch.n_cce, nt, dev.get("cce_q"), dev.get("cce_sf"), dev.get("cce_cb"),
                         dev.get("cce_ics"), _ptr(batch.cce_terms), _ptr(batch._status()))
        self._check(lib().jaad_decode_batch_device(self.h, C.byref(bs), pcm_dev_ptr, pcm_bytes, flags, stream_ptr),
                    "jaad_decode_batch_device")

    def state_export(self, slot: int) -> np.ndarray:
        n = lib().jaad_state_bytes(self.h)
        buf = np.empty(n, np.uint8)
        self._check(lib().jaad_state_export(self.h, slot, _ptr(buf), n), "jaad_state_export")
        return buf

    def state_import(self, slot: int, buf: np.ndarray) -> None:
        buf = np.ascontiguousarray(buf, np.uint8)
        self._check(lib().jaad_state_import(self.h, slot, _ptr(buf), buf.nbytes), "jaad_state_import")

    def state_reset(self, slot: int) -> None:
        self._check(lib().jaad_state_reset(self.h, slot), "jaad_state_reset")


# ---------------------------------------------------------------------------------------------
# host bitstream front end (include/jaad_parse.h)
# ---------------------------------------------------------------------------------------------
def asc_parse(asc: bytes) -> StreamCfg:
    """AudioSpecificConfig -> StreamCfg (DecoderConfig.decode, A/DecoderConfig.java:175-291)."""
    cfg = StreamCfg()
    rc = lib().jaad_asc_parse(bytes(asc), len(asc), C.byref(cfg))
    if rc:
        raise JaadError(rc, "jaad_asc_parse")
    return cfg


def adts_frames(data: bytes):
    """Split an ADTS byte stream (S/adts/ADTSDemultiplexer.java): yields (header, raw_data_block)."""
    pos = 0
    h = AdtsHeader()
    off = C.c_size_t()
    data = bytes(data)
    base = C.cast(C.c_char_p(data), C.c_void_p).value  # one buffer, searched at an offset (no copies)
    while pos < len(data):
        rc = lib().jaad_adts_find(C.c_void_p(base + pos), len(data) - pos, C.byref(off), C.byref(h))
        if rc == ERR_EOS:
            return
        if rc:
            raise JaadError(rc, "jaad_adts_find")
        start = pos + off.value + h.header_bytes
        end = pos + off.value + h.frame_length
        if h.frame_length < h.header_bytes or end > len(data):
            return  # truncated last frame (EOF inside the payload)
        yield AdtsHeader.from_buffer_copy(h), data[start:end]
        pos = end


def raw_pce_cfg(raw: bytes) -> StreamCfg:
    """The configuration a raw_data_block's leading PCE declares (jaad_raw_pce_cfg)."""
    cfg = StreamCfg()
    rc = lib().jaad_raw_pce_cfg(bytes(raw), len(raw), C.byref(cfg))
    if rc:
        raise JaadError(rc, "jaad_raw_pce_cfg")
    return cfg


def adts_cfg(h: AdtsHeader) -> StreamCfg:
    cfg = StreamCfg()
    rc = lib().jaad_adts_cfg(C.byref(h), C.byref(cfg))
    if rc:
        raise JaadError(rc, "jaad_adts_cfg")
    return cfg


def probe_sbr(cfg: StreamCfg, frame: bytes) -> bool:
    """Does this raw_data_block of a core configuration carry an SBR payload (implicit SBR)?"""
    found = C.c_uint32()
    rc = lib().jaad_probe_sbr(C.byref(cfg), bytes(frame), len(frame), C.byref(found))
    if rc:
        raise JaadError(rc, "jaad_probe_sbr")
    return bool(found.value & 1)


def implicit_sbr_cfg(cfg: StreamCfg, from_asc: bool = False) -> StreamCfg:
    """The configuration the reference switches to when it meets SBR data in a core stream
    (DecoderConfig.setSBRPresent, A/DecoderConfig.java:124-135): a mono core decodes to stereo
    (SCE.isStereo) with PS applied when present (psEnabled).  The output rate is doubled for a
    decoder created from an ADTS header (AudioDecoderInfo: outputFrequency unset) unless
    SampleFrequency.duplicated() is SF_NONE (above 48 kHz); a decoder created from an
    AudioSpecificConfig already has outputFrequency = the core rate (A/DecoderConfig.java:180),
    so its SBR runs downsampled at the core rate (A/sbr/SBR.java:100)."""
    return make_cfg(cfg.sf_index, cfg.channel_config, cfg.tns_mode, sbr=True, ps=cfg.channel_config == 1,
                    down=from_asc or cfg.sf_index < 3)


class Parser:
    """One stream's host parser state (window shapes, static PNS LCG, SBR/PS history)."""

    def __init__(self, cfg: StreamCfg):
        self.cfg = cfg
        self.nch = core_channels(cfg)
        h = C.c_void_p()
        rc = lib().jaad_parser_create(C.byref(cfg), C.byref(h))
        if rc:
            raise JaadError(rc, "jaad_parser_create")
        self.h = h

    def close(self):
        h = getattr(self, "h", None)
        if h:
            self.h = None
            lib().jaad_parser_destroy(h)

    def __del__(self):
        try:
            self.close()
        except TypeError:  # interpreter shutdown (see Context.__del__)
            pass

    def snapshot(self) -> "Parser":
        """A copy of the whole parser state (jaad_parser_clone)."""
        h = C.c_void_p()
        rc = lib().jaad_parser_clone(self.h, C.byref(h))
        if rc:
            raise JaadError(rc, "jaad_parser_clone")
        s = Parser.__new__(Parser)
        s.cfg, s.nch, s.h = self.cfg, self.nch, h
        return s

    def restore(self, snap: "Parser") -> None:
        """Roll the state back to a snapshot (jaad_parser_copy)."""
        rc = lib().jaad_parser_copy(self.h, snap.h)
        if rc:
            raise JaadError(rc, "jaad_parser_copy")

    @property
    def pns_state(self) -> int:
        return int(lib().jaad_parser_pns_state(self.h))

    @pns_state.setter
    def pns_state(self, v: int) -> None:
        lib().jaad_parser_set_pns_state(self.h, v)

    def parse(self, frames: list, slot: int = 0, drop_eos: bool = False) -> Batch:
        """raw_data_blocks (bytes) of this stream -> one-run Batch in the jaad_gpu.h layout.

        drop_eos: a frame whose bitstream ends early (JAAD_ERR_EOS) is marked FRAME_EOS in
        batch.frame_status -- the decode then drops it as Decoder.decodeFrame drops a frame that
        throws EOSException (A/Decoder.java:89-101) -- and parsing goes on with the next frame
        (from the state the truncated frame left: window shapes and the PNS LCG moved as far as
        the reference's reads got before its EOSException, jaad_parse.h).  Without it the
        JaadError propagates."""
        nf, nch, ncpe = len(frames), self.nch, n_cpe(self.cfg)
        status = None
        q = np.zeros((nf * nch, 1024), np.int16)
        sf = np.zeros((nf * nch, 128), np.uint8)
        cb = np.zeros((nf * nch, 128), np.uint8)
        ics = np.zeros(nf * nch, ICS_DTYPE)
        ms = np.zeros((nf, 2 * ncpe), np.uint64) if ncpe else None
        tns = np.zeros(nf * nch, TNS_DTYPE)
        ne = n_elements(self.cfg)
        sbr = np.zeros((nf, ne) if ne > 1 else nf, SBR_FRAME_DTYPE) if self.cfg.sbr else None
        # coupling channel elements: up to 8 records and 64 terms per frame
        cq = np.zeros((8, 1024), np.int16)
        csf = np.zeros((8, 128), np.uint8)
        ccb = np.zeros((8, 128), np.uint8)
        cics = np.zeros(8, ICS_DTYPE)
        cterms = np.zeros(64, CCE_TERM_DTYPE)
        recs, terms = [], []
        for i, fr in enumerate(frames):
            o = FrameOut(q[i * nch:].ctypes.data, sf[i * nch:].ctypes.data, cb[i * nch:].ctypes.data,
                         ics[i * nch:].ctypes.data, ms[i:].ctypes.data if ms is not None else None,
                         tns[i * nch:].ctypes.data, sbr[i:].ctypes.data if sbr is not None else None,
                         cq.ctypes.data, csf.ctypes.data, ccb.ctypes.data, cics.ctypes.data, cterms.ctypes.data,
                         8, 64, 0, 0)
            rc = lib().jaad_parse_frame(self.h, bytes(fr), len(fr), C.byref(o))
            if rc == ERR_EOS and drop_eos:
                if status is None:
                    status = np.zeros(nf, np.uint8)
                status[i] = FRAME_EOS
                for a in (q, sf, cb, ics, tns):
                    a[i * nch:(i + 1) * nch] = 0
                if ms is not None:
                    ms[i] = 0
                # the SBR records stay as the parser left them: an SBR payload read whole before
                # the bitstream ended keeps its header, which the reference swapped in before the
                # EOSException (A/sbr/SBR.java:162-184) and the DSP stage applies (zero otherwise)
                continue
            if rc:
                raise JaadError(rc, f"jaad_parse_frame (frame {i})")
            if o.n_cce:
                if len(recs) + o.n_cce > CCE_MAX_RECORDS:  # jaad_cce_term.cce is 16-bit (jaad_gpu.h)
                    raise JaadError(ERR_UNSUPPORTED, f"more than {CCE_MAX_RECORDS} CCE records in one batch "
                                                     f"(frame {i}): parse fewer frames per call")
                t = cterms[:o.n_cce_terms].copy()
                t["frame"] = i
                t["cce"] += len(recs)
                terms.append(t)
                recs += [(cq[k].copy(), csf[k].copy(), ccb[k].copy(), cics[k].copy()) for k in range(o.n_cce)]
        if not (ics["flags"] & ICS_TNS).any():
            tns = None
        b = Batch(q, sf, cb, ics, ms, tns, np.array([slot], np.uint32), np.array([0, nf], np.uint32), nch)
        b.sbr = sbr
        b.frame_status = status
        if recs:
            b.cce_q = np.ascontiguousarray(np.stack([r[0] for r in recs]))
            b.cce_sf = np.ascontiguousarray(np.stack([r[1] for r in recs]))
            b.cce_cb = np.ascontiguousarray(np.stack([r[2] for r in recs]))
            b.cce_ics = np.ascontiguousarray(np.array([r[3] for r in recs], ICS_DTYPE))
            b.cce_terms = np.ascontiguousarray(np.concatenate(terms)) if terms else np.zeros(0, CCE_TERM_DTYPE)
        return b
