"""The JNI glue (jaadec_amd/csrc/jaad_jni.c) compiled against a mock JNIEnv
(tests/jni_mock/): its argument and capacity checks and its AACException mapping run here
without a JDK; with a GPU the same entry points decode a batch through direct buffers."""
import ctypes as C
from pathlib import Path

import numpy as np
import pytest

from jaadec_amd import native as N

LIB = Path(__file__).resolve().parent / "jni_mock" / "libjaadjni_mock.so"
PFX = "Java_net_sourceforge_jaad_aac_gpu_GpuDSP_"
AAC_EXC = "net/sourceforge/jaad/aac/AACException"


class Buf(C.Structure):
    """A mock direct ByteBuffer: (address, capacity)."""
    _fields_ = [("address", C.c_void_p), ("capacity", C.c_int64)]


def _lib():
    if not LIB.exists():
        pytest.skip("libjaadjni_mock.so not built (python -m jaadec_amd.build)")
    L = C.CDLL(str(LIB))
    L.jni_mock_env.restype = C.c_void_p
    L.jni_mock_take_exception.argtypes = [C.c_char_p, C.c_int, C.c_char_p, C.c_int]
    create = getattr(L, PFX + "nativeCreate")
    create.argtypes = [C.c_void_p, C.c_void_p] + [C.c_int32] * 8
    create.restype = C.c_int64
    getattr(L, PFX + "nativeDestroy").argtypes = [C.c_void_p, C.c_void_p, C.c_int64]
    decode = getattr(L, PFX + "nativeDecode")
    decode.argtypes = ([C.c_void_p, C.c_void_p, C.c_int64, C.c_int32, C.c_int32, C.c_int32] + [C.c_void_p] * 10 +
                       [C.c_int32, C.c_void_p])
    getattr(L, PFX + "nativeReset").argtypes = [C.c_void_p, C.c_void_p, C.c_int64, C.c_int32]
    for name in ("nativeRegister", "nativeUnregister", "nativeFreeDirect"):
        getattr(L, PFX + name).argtypes = [C.c_void_p, C.c_void_p, C.c_int64, C.c_void_p]
    coupled = getattr(L, PFX + "nativeDecodeCoupled")
    coupled.argtypes = ([C.c_void_p, C.c_void_p, C.c_int64, C.c_int32, C.c_int32, C.c_int32] + [C.c_void_p] * 10 +
                        [C.c_int32, C.c_int32, C.c_int32] + [C.c_void_p] * 6)
    getattr(L, PFX + "nativeStateBytes").argtypes = [C.c_void_p, C.c_void_p, C.c_int64]
    getattr(L, PFX + "nativeStateBytes").restype = C.c_int32
    for name in ("nativeStateExport", "nativeStateImport"):
        getattr(L, PFX + name).argtypes = [C.c_void_p, C.c_void_p, C.c_int64, C.c_int32, C.c_void_p]
    alloc = getattr(L, PFX + "nativeAllocDirect")
    alloc.argtypes = [C.c_void_p, C.c_void_p, C.c_int64, C.c_int64]
    alloc.restype = C.c_void_p
    return L


def _exception(L):
    cls, msg = C.create_string_buffer(256), C.create_string_buffer(1024)
    if not L.jni_mock_take_exception(cls, 256, msg, 1024):
        return None
    return cls.value.decode(), msg.value.decode()


def _buf(a, keep):
    if a is None:
        return None
    b = Buf(a.ctypes.data, a.nbytes)
    keep.append(b)
    return C.addressof(b)


def test_exports():
    L = _lib()
    for name in ("nativeCreate", "nativeDestroy", "nativeDecode", "nativeReset", "nativeRegister",
                 "nativeUnregister", "nativeAllocDirect", "nativeFreeDirect", "nativeDecodeCoupled",
                 "nativeStateBytes", "nativeStateExport", "nativeStateImport"):
        assert hasattr(L, PFX + name)


def test_invalid_handles_throw_aac_exception():
    L = _lib()
    env = L.jni_mock_env()
    getattr(L, PFX + "nativeDecode")(env, None, 0, 1, 1, 2, *([None] * 10), 0, None)
    cls, msg = _exception(L)
    assert cls == AAC_EXC and N.strerror(N.ERR_INVALID_ARG) in msg
    getattr(L, PFX + "nativeReset")(env, None, 0, 0)
    cls, msg = _exception(L)
    assert cls == AAC_EXC and N.strerror(N.ERR_INVALID_ARG) in msg
    getattr(L, PFX + "nativeDestroy")(env, None, 0)  # a null handle is a no-op
    assert _exception(L) is None
    a = np.zeros(64, np.uint8)
    b = Buf(a.ctypes.data, a.nbytes)
    for name in ("nativeRegister", "nativeUnregister", "nativeFreeDirect"):
        getattr(L, PFX + name)(env, None, 0, C.addressof(b))
        cls, msg = _exception(L)
        assert cls == AAC_EXC and N.strerror(N.ERR_INVALID_ARG) in msg
    assert getattr(L, PFX + "nativeAllocDirect")(env, None, 0, 4096) is None
    cls, msg = _exception(L)
    assert cls == AAC_EXC and N.strerror(N.ERR_INVALID_ARG) in msg
    assert getattr(L, PFX + "nativeStateBytes")(env, None, 0) == 0
    cls, msg = _exception(L)
    assert cls == AAC_EXC and N.strerror(N.ERR_INVALID_ARG) in msg
    for name in ("nativeStateExport", "nativeStateImport"):
        getattr(L, PFX + name)(env, None, 0, 0, C.addressof(b))
        cls, msg = _exception(L)
        assert cls == AAC_EXC and N.strerror(N.ERR_INVALID_ARG) in msg


def test_create_without_gpu_throws_no_device():
    import torch
    if torch.cuda.device_count() > 0:
        pytest.skip("a GPU is present")
    L = _lib()
    h = getattr(L, PFX + "nativeCreate")(L.jni_mock_env(), None, 3, 2, 0, 0, 0, 0, 4, 0)
    assert h == 0
    cls, msg = _exception(L)
    assert cls == AAC_EXC and N.strerror(N.ERR_NO_DEVICE) in msg


@pytest.mark.gpu
def test_decode_through_direct_buffers_and_capacity_checks():
    L = _lib()
    env = L.jni_mock_env()
    p = N.synth_params(2, n_streams=3, frames_per_stream=20)
    b = N.synth_batch(p)
    with N.Context(N.make_cfg(), 3) as ctx:
        want = ctx.decode(b, N.PCM_BIG_ENDIAN)
    h = getattr(L, PFX + "nativeCreate")(env, None, 3, 2, 0, 0, 0, 0, 3, 0)
    assert h and _exception(L) is None
    decode = getattr(L, PFX + "nativeDecode")
    try:
        out = np.zeros_like(want)
        keep = []
        args = [_buf(x, keep) for x in (b.stream_slot, b.frame_begin, b.q, b.sf, b.cb, b.ics, b.ms_used, b.tns, None,
                                         out)]
        decode(env, None, h, b.n_frames, len(b.stream_slot), 2, *args, N.PCM_BIG_ENDIAN, None)
        assert _exception(L) is None
        assert (out == want).all()
        # the same buffers page-locked once (nativeRegister): DMA without staging, same PCM
        reg = [a for a in (args[2], args[3], args[4], args[5], args[6], args[9])]
        for r in reg:
            getattr(L, PFX + "nativeRegister")(env, None, h, r)
            assert _exception(L) is None
        out[:] = 0
        for slot in range(3):  # from fresh stream states again
            getattr(L, PFX + "nativeReset")(env, None, h, slot)
        decode(env, None, h, b.n_frames, len(b.stream_slot), 2, *args, N.PCM_BIG_ENDIAN, None)
        assert _exception(L) is None
        assert (out == want).all()
        for r in reg:
            getattr(L, PFX + "nativeUnregister")(env, None, h, r)
            assert _exception(L) is None
        # nch must be the context's channels per record
        decode(env, None, h, b.n_frames, len(b.stream_slot), 1, *args, N.PCM_BIG_ENDIAN, None)
        cls, msg = _exception(L)
        assert cls == AAC_EXC and N.strerror(N.ERR_INVALID_ARG) in msg
        # a q buffer one ch-frame short is refused before any copy
        short = list(args)
        qshort = Buf(b.q.ctypes.data, b.q.nbytes - 2048)
        keep.append(qshort)
        short[2] = C.addressof(qshort)
        decode(env, None, h, b.n_frames, len(b.stream_slot), 2, *short, N.PCM_BIG_ENDIAN, None)
        cls, msg = _exception(L)
        assert cls == AAC_EXC and N.strerror(N.ERR_INVALID_ARG) in msg
        # a PCM buffer too small for the batch
        small = np.zeros(want.nbytes - 1, np.uint8)
        args2 = list(args)
        args2[9] = _buf(small, keep)
        decode(env, None, h, b.n_frames, len(b.stream_slot), 2, *args2, N.PCM_BIG_ENDIAN, None)
        cls, msg = _exception(L)
        assert cls == AAC_EXC and N.strerror(N.ERR_INVALID_ARG) in msg
        # a bitstream error (max_sfb beyond the swb count) maps to AACException too
        bad = b.ics.copy()
        bad["max_sfb"][0] = 60
        args3 = list(args)
        args3[5] = _buf(bad, keep)
        decode(env, None, h, b.n_frames, len(b.stream_slot), 2, *args3, N.PCM_BIG_ENDIAN, None)
        cls, msg = _exception(L)
        assert cls == AAC_EXC and N.strerror(N.ERR_BITSTREAM) in msg
        getattr(L, PFX + "nativeReset")(env, None, h, 1)
        assert _exception(L) is None
        # PCM into a direct buffer over context-owned page-locked memory (nativeAllocDirect)
        db = getattr(L, PFX + "nativeAllocDirect")(env, None, h, want.nbytes)
        assert db and _exception(L) is None
        mb = Buf.from_address(db)
        assert mb.capacity == want.nbytes
        args4 = list(args)
        args4[9] = db
        for slot in range(3):
            getattr(L, PFX + "nativeReset")(env, None, h, slot)
        decode(env, None, h, b.n_frames, len(b.stream_slot), 2, *args4, N.PCM_BIG_ENDIAN, None)
        assert _exception(L) is None
        got = np.ctypeslib.as_array((C.c_uint8 * want.nbytes).from_address(mb.address)).reshape(want.shape)
        assert (got == want).all()
        getattr(L, PFX + "nativeFreeDirect")(env, None, h, db)
        assert _exception(L) is None
        getattr(L, PFX + "nativeFreeDirect")(env, None, h, db)  # freed already
        cls, msg = _exception(L)
        assert cls == AAC_EXC and N.strerror(N.ERR_INVALID_ARG) in msg
    finally:
        getattr(L, PFX + "nativeDestroy")(env, None, h)


@pytest.mark.gpu
def test_coupled_decode_through_direct_buffers():
    """nativeDecodeCoupled: a stereo batch with CCE records and terms equals the Python entry."""
    from tests.test_cce import coupled_batch
    L = _lib()
    env = L.jni_mock_env()
    b = coupled_batch(2, n_streams=2, fps=12, seed=4)
    with N.Context(N.make_cfg(), 2) as ctx:
        want = ctx.decode(b, N.PCM_BIG_ENDIAN)
    h = getattr(L, PFX + "nativeCreate")(env, None, 3, 2, 0, 0, 0, 0, 2, 0)
    assert h and _exception(L) is None
    try:
        out = np.zeros_like(want)
        keep = []
        a = [_buf(x, keep) for x in (b.stream_slot, b.frame_begin, b.q, b.sf, b.cb, b.ics, b.ms_used, None, None,
                                     out)]
        c = [_buf(x, keep) for x in (b.cce_q, b.cce_sf, b.cce_cb, b.cce_ics, b.cce_terms)]
        getattr(L, PFX + "nativeDecodeCoupled")(env, None, h, b.n_frames, len(b.stream_slot), 2, *a, N.PCM_BIG_ENDIAN,
                                               b.n_cce, len(b.cce_terms), *c, None)
        assert _exception(L) is None
        assert (out == want).all()
        # a term buffer one term short is refused
        short = Buf(b.cce_terms.ctypes.data, b.cce_terms.nbytes - 488)
        keep.append(short)
        c[4] = C.addressof(short)
        getattr(L, PFX + "nativeDecodeCoupled")(env, None, h, b.n_frames, len(b.stream_slot), 2, *a, N.PCM_BIG_ENDIAN,
                                               b.n_cce, len(b.cce_terms), *c, None)
        cls, msg = _exception(L)
        assert cls == AAC_EXC and N.strerror(N.ERR_INVALID_ARG) in msg
    finally:
        getattr(L, PFX + "nativeDestroy")(env, None, h)


@pytest.mark.gpu
def test_coupled_he_aac_v2_decode_through_direct_buffers():
    """nativeDecodeCoupled with an sbr buffer: an HE-AAC v2 batch (mono core + PS) whose frames carry
    coupling terms on the core channel equals the Python entry, PCM for PCM."""
    from tests.test_cce import cce_records
    L = _lib()
    env = L.jni_mock_env()
    p = N.synth_params(5, n_streams=3, frames_per_stream=16)
    b = N.synth_batch(p)
    cfg = N.cfg_for(p)
    rng = np.random.default_rng(23)
    n_rec = 8
    b.cce_q, b.cce_sf, b.cce_cb, b.cce_ics = cce_records(n_rec, 23, pns=10, sf_index=p.sf_index)
    terms = []
    for f in range(b.n_frames):
        if rng.integers(2):
            continue
        t = np.zeros((), N.CCE_TERM_DTYPE)
        t["frame"], t["channel"], t["point"], t["cce"] = f, 0, rng.integers(2), rng.integers(n_rec)
        t["gain"] = rng.choice([0.0, 1.0, -0.5, 2.0, 1.0905077], 120).astype(np.float32)
        terms.append(t)
    b.cce_terms = np.array(terms, N.CCE_TERM_DTYPE)
    with N.Context(cfg, 3) as ctx:
        want = ctx.decode(b, N.PCM_BIG_ENDIAN)
    h = getattr(L, PFX + "nativeCreate")(env, None, p.sf_index, p.channel_config, 0, 1, 1, 0, 3, 0)
    assert h and _exception(L) is None
    try:
        out = np.zeros_like(want)
        keep = []
        a = [_buf(x, keep) for x in (b.stream_slot, b.frame_begin, b.q, b.sf, b.cb, b.ics, None, b.tns, b.sbr, out)]
        c = [_buf(x, keep) for x in (b.cce_q, b.cce_sf, b.cce_cb, b.cce_ics, b.cce_terms)]
        getattr(L, PFX + "nativeDecodeCoupled")(env, None, h, b.n_frames, len(b.stream_slot), 1, *a, N.PCM_BIG_ENDIAN,
                                               b.n_cce, len(b.cce_terms), *c, None)
        assert _exception(L) is None
        assert (out == want).all()
        # an sbr buffer one frame short is refused before any copy
        short = Buf(b.sbr.ctypes.data, b.sbr.nbytes - b.sbr.itemsize)
        keep.append(short)
        a[8] = C.addressof(short)
        getattr(L, PFX + "nativeDecodeCoupled")(env, None, h, b.n_frames, len(b.stream_slot), 1, *a, N.PCM_BIG_ENDIAN,
                                               b.n_cce, len(b.cce_terms), *c, None)
        cls, msg = _exception(L)
        assert cls == AAC_EXC and N.strerror(N.ERR_INVALID_ARG) in msg
    finally:
        getattr(L, PFX + "nativeDestroy")(env, None, h)


@pytest.mark.gpu
def test_lsb1_precision_through_the_jni_create():
    """nativeCreate's precision argument reaches jaad_stream_cfg.precision: JAAD_PRECISION_LSB1 decodes
    the stereo batch the same as the Python entry's LSB1 context (within 1 LSB of the exact PCM, and
    not identical to it); a value other than 0 / 1 is refused at create."""
    L = _lib()
    env = L.jni_mock_env()
    p = N.synth_params(2, n_streams=3, frames_per_stream=20)
    b = N.synth_batch(p)
    with N.Context(N.make_cfg(precision=N.PRECISION_LSB1), 3) as ctx:
        want = ctx.decode(b, N.PCM_BIG_ENDIAN)
    with N.Context(N.make_cfg(), 3) as ctx:
        exact = ctx.decode(b, N.PCM_BIG_ENDIAN)
    h = getattr(L, PFX + "nativeCreate")(env, None, 3, 2, 0, 0, 0, N.PRECISION_LSB1, 3, 0)
    assert h and _exception(L) is None
    try:
        out = np.zeros_like(want)
        keep = []
        args = [_buf(x, keep) for x in (b.stream_slot, b.frame_begin, b.q, b.sf, b.cb, b.ics, b.ms_used, b.tns, None,
                                         out)]
        getattr(L, PFX + "nativeDecode")(env, None, h, b.n_frames, len(b.stream_slot), 2, *args, N.PCM_BIG_ENDIAN, None)
        assert _exception(L) is None
        assert (out == want).all()
        d = np.abs(out.view(">i2").astype(np.int32) - exact.view(">i2").astype(np.int32))
        assert d.max() == 1
    finally:
        getattr(L, PFX + "nativeDestroy")(env, None, h)
    assert not getattr(L, PFX + "nativeCreate")(env, None, 3, 2, 0, 0, 0, 2, 3, 0)
    cls, msg = _exception(L)
    assert cls == AAC_EXC
