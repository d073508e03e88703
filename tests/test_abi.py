"""The C-ABI library (no compute calls: this runs without a GPU)."""
import ctypes as C
import re
import subprocess
from pathlib import Path

import pytest

from jaadec_amd import native as N

ROOT = Path(__file__).resolve().parents[1]


def header_functions(path):
    src = Path(path).read_text()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"^\s*(?:const\s+)?[a-z_0-9]+\s*\*?\s*(jaad_[a-z_0-9]+)\s*\(", src, re.M)))


def test_library_exports_every_header_symbol():
    lib = N.lib()
    declared = header_functions(ROOT / "include" / "jaad_gpu.h")
    assert set(declared) == set(N.EXPORTS), declared
    for name in declared:
        assert hasattr(lib, name), name


@pytest.mark.parametrize("header", ["jaad_parse.h", "jaad_mp4.h"])
def test_library_exports_the_front_end_headers(header):
    """The host front end (bitstream parser, MP4 feeder) lives in the same library."""
    lib = N.lib()
    declared = header_functions(ROOT / "include" / header)
    assert declared
    for name in declared:
        assert hasattr(lib, name), name


def test_exported_dynamic_symbols_with_nm():
    out = subprocess.run(["nm", "-D", "--defined-only", str(N.LIB_PATH)], capture_output=True, text=True).stdout
    syms = {line.split()[-1] for line in out.splitlines() if line.strip()}
    for name in header_functions(ROOT / "include" / "jaad_gpu.h"):
        assert name in syms


def test_synth_library_exports():
    s = N.synth_lib()
    for name in header_functions(ROOT / "include" / "jaad_synth.h"):
        assert hasattr(s, name)


def test_strerror_and_status_codes():
    assert N.strerror(N.OK) == "ok"
    assert "device" in N.strerror(N.ERR_NO_DEVICE)
    assert N.strerror(-99) == "unknown status"


def test_config_queries_mirror_decoderconfig():
    cfg = N.make_cfg(sf_index=4, channel_config=1)
    L = N.lib()
    assert L.jaad_cfg_sample_length(C.byref(cfg)) == 1024
    assert L.jaad_cfg_channel_count(C.byref(cfg)) == 2  # mono -> stereo while sbrEnabled
    assert L.jaad_frame_pcm_bytes(C.byref(cfg), N.PCM_BIG_ENDIAN) == 4096
    assert L.jaad_frame_pcm_bytes(C.byref(cfg), N.PCM_FLOAT32) == 8192
    up = N.make_cfg(sf_index=6, channel_config=2, sbr=True)
    down = N.make_cfg(sf_index=6, channel_config=2, sbr=True, down=True)
    assert L.jaad_cfg_sample_length(C.byref(up)) == 2048   # upsampling SBR doubles the length
    assert L.jaad_cfg_sample_length(C.byref(down)) == 1024  # downsampled SBR keeps the core rate
    for cc, n in ((3, 3), (4, 4), (5, 5), (6, 6), (7, 8)):  # ChannelConfiguration: 5.1 = 6, 7.1 = 8
        mc = N.make_cfg(channel_config=cc)
        assert L.jaad_cfg_channel_count(C.byref(mc)) == n
        assert L.jaad_frame_pcm_bytes(C.byref(mc), N.PCM_BIG_ENDIAN) == 1024 * n * 2
    # multichannel HE-AAC: SCE and CPE give two channels each, the LFE one (SCE.java:115-132)
    for cc, n in ((3, 4), (4, 6), (5, 6), (6, 7), (7, 9)):
        mc = N.make_cfg(sf_index=6, channel_config=cc, sbr=True)
        assert L.jaad_cfg_channel_count(C.byref(mc)) == n == N.out_channels(mc)
        assert L.jaad_frame_pcm_bytes(C.byref(mc), N.PCM_FLOAT32) == 2048 * n * 4


@pytest.mark.parametrize("fields,status", [
    ({"abi_version": 99}, N.ERR_ABI),
    ({"profile": 1}, N.ERR_UNSUPPORTED),      # AAC Main: ICPrediction is out of scope
    ({"sf_index": 12}, N.ERR_UNSUPPORTED),
    ({"channel_config": 8}, N.ERR_UNSUPPORTED),               # no configuration 8
    ({"channel_config": 6, "sbr": 1, "ps": 1, "ext_sf_index": 0}, N.ERR_UNSUPPORTED),  # PS: mono streams only
    ({"sbr": 1, "ext_sf_index": 1}, N.ERR_UNSUPPORTED),    # SBR output rate must be 2x the core rate
    ({"sbr": 1, "sf_index": 1, "ext_sf_index": 0}, N.ERR_UNSUPPORTED),
    ({"ps": 1, "sbr": 1, "channel_config": 2}, N.ERR_UNSUPPORTED),  # PS needs an SCE core
])
def test_ctx_create_rejects_bad_config(fields, status):
    cfg = N.make_cfg()
    for field, value in fields.items():
        setattr(cfg, field, value)
    h = C.c_void_p()
    assert N.lib().jaad_ctx_create(C.byref(cfg), 4, 0, C.byref(h)) == status
    assert not h.value


def test_ctx_create_without_gpu_fails_loudly():
    """No silent CPU fallback: without a gfx950 device the product path refuses to run."""
    from conftest import gpu_available
    if gpu_available():
        pytest.skip("a GPU is present")
    with pytest.raises(N.JaadError) as e:
        N.Context(N.make_cfg(), 4)
    assert e.value.status == N.ERR_NO_DEVICE


def test_null_arguments_are_rejected():
    L = N.lib()
    assert L.jaad_ctx_create(None, 4, 0, None) == N.ERR_INVALID_ARG
    assert L.jaad_decode_batch(None, None, None, 0, 0) == N.ERR_INVALID_ARG
    assert L.jaad_state_reset(None, 0) == N.ERR_INVALID_ARG
    L.jaad_ctx_destroy(None)  # no-op


def test_jni_glue_matches_java_natives_in_integration_doc():
    """Every `native` method of the GpuDSP class shown in INTEGRATION.md has a JNI symbol in jaad_jni.c."""
    doc = (ROOT / "INTEGRATION.md").read_text()
    natives = set(re.findall(r"private static native \w+ (\w+)\(", doc))
    glue = (ROOT / "jaadec_amd" / "csrc" / "jaad_jni.c").read_text()
    defined = set(re.findall(r"Java_net_sourceforge_jaad_aac_gpu_GpuDSP_(\w+)\(", glue))
    assert natives and natives == defined
    for fn in re.findall(r"\b(jaad_[a-z_]+)\(", glue):
        assert fn in N.EXPORTS, fn
