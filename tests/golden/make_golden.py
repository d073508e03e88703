"""Generate the committed fixtures in tests/golden/ (inputs + expected PCM).

The expected outputs come from the C restatement of the reference DSP (oracle/), because the
reference itself (Java) cannot be run in this image and ships no vectors of its own (SURVEY.md
s4, s8c).  The fixtures pin the restatement, the synthetic-input generator and the HIP path
against silent drift; their relation to the Java code rests on tests/test_oracle.py.

    python tests/golden/make_golden.py
"""
import sys
from pathlib import Path

import numpy as np

HERE = Path(__file__).resolve().parent
sys.path.insert(0, str(HERE.parents[1]))
from jaadec_amd import native as N  # noqa: E402
from oracle import oracle as O  # noqa: E402

CASES = {
    # name: (config id, overrides, cfg kwargs, flags)
    "c1_mono_44k_one_frame": (1, dict(), dict(sf_index=4, channel_config=1), N.PCM_BIG_ENDIAN),
    "c2_stereo_48k_long": (2, dict(n_streams=2, frames_per_stream=5), dict(), N.PCM_BIG_ENDIAN),
    "c3_switching_tns_compat": (3, dict(n_streams=2, frames_per_stream=12), dict(), N.PCM_BIG_ENDIAN),
    "c3_switching_tns_spec_f32": (3, dict(n_streams=2, frames_per_stream=10), dict(tns_mode=N.TNS_SPEC), N.PCM_FLOAT32),
    "pns_is_le": (3, dict(n_streams=2, frames_per_stream=8, pns_percent=10, is_percent=20), dict(), N.PCM_LITTLE_ENDIAN),
    # HE-AAC: SBR records (jaad_sbr_frame) ride along; cfg from the synthetic parameters
    "c4_sbr_stereo_f32": (4, dict(n_streams=2, frames_per_stream=6), None, N.PCM_FLOAT32),
    "c5_sbr_ps_be": (5, dict(n_streams=2, frames_per_stream=6), None, N.PCM_BIG_ENDIAN),
}


def save(name, cfgid, over, cfgkw, flags):
    p = N.synth_params(cfgid, **over)
    b = N.synth_batch(p)
    if cfgkw is None:
        cfg = N.cfg_for(p)
    else:
        cfg = N.make_cfg(**{"sf_index": p.sf_index, "channel_config": p.channel_config, **cfgkw})
    pcm = O.decode_batch(cfg, b, O.Streams(int(b.stream_slot.max()) + 1), flags)
    arrays = dict(q=b.q, sf=b.sf, cb=b.cb, ics=b.ics.view(np.uint8), stream_slot=b.stream_slot,
                  frame_begin=b.frame_begin, pcm=pcm,
                  meta=np.array([cfg.sf_index, cfg.channel_config, cfg.tns_mode, flags, b.nch,
                                 cfg.sbr, cfg.ps, cfg.ext_sf_index], np.int32))
    if b.sbr is not None:
        arrays["sbr"] = b.sbr.view(np.uint8)
    if b.ms_used is not None:
        arrays["ms_used"] = b.ms_used
    if b.tns is not None:
        arrays["tns"] = b.tns.view(np.uint8)
    np.savez_compressed(HERE / f"{name}.npz", **arrays)
    print(name, b.n_frames, "frames", pcm.nbytes, "PCM bytes")


# bitstream fixtures: the synthetic records written as raw_data_blocks / an ADTS stream by the
# test writer (oracle/jaad_writer.c); expected PCM = the restatement's decode of those records
BITSTREAMS = {
    # name: (config id, overrides, container, writer extras)
    "c1_raw_frame": (1, dict(), "raw", 0),
    "c3_adts_stream": (3, dict(n_streams=1, frames_per_stream=24, pns_percent=5, is_percent=10), "adts", 3),
}


def save_bitstream(name, cfgid, over, container, extras):
    p = N.synth_params(cfgid, **over)
    b = N.synth_batch(p)
    cfg = N.make_cfg(sf_index=p.sf_index, channel_config=p.channel_config)
    frames = O.write_frames(b, p.sf_index, extras=extras)
    data = frames[0] if container == "raw" else O.adts_wrap(frames, p.sf_index, p.channel_config)
    pcm = O.decode_batch(cfg, b, O.Streams(1), N.PCM_BIG_ENDIAN)
    np.savez_compressed(HERE / f"{name}.npz", data=np.frombuffer(data, np.uint8), pcm=pcm,
                        meta=np.array([p.sf_index, p.channel_config, int(b.ics["pns_state"][0]),
                                       len(frames)], np.int64))
    print(name, len(frames), "frames", len(data), "bytes")


def load(path):
    z = np.load(path, allow_pickle=False)
    meta = [int(v) for v in z["meta"]] + [0, 0, 0]
    sf_index, ch, tns_mode, flags, nch, sbr, ps, ext_sf = meta[:8]
    b = N.Batch(z["q"], z["sf"], z["cb"], z["ics"].view(N.ICS_DTYPE).reshape(-1),
                z["ms_used"] if "ms_used" in z else None,
                z["tns"].view(N.TNS_DTYPE).reshape(-1) if "tns" in z else None,
                z["stream_slot"], z["frame_begin"], nch,
                z["sbr"].view(N.SBR_FRAME_DTYPE).reshape(-1) if "sbr" in z else None)
    cfg = N.make_cfg(sf_index=sf_index, channel_config=ch, tns_mode=tns_mode, sbr=bool(sbr), ps=bool(ps))
    assert cfg.ext_sf_index == ext_sf
    return b, cfg, flags, z["pcm"]


if __name__ == "__main__":
    for k, v in CASES.items():
        if len(sys.argv) > 1 and k not in sys.argv[1:]:
            continue
        save(k, *v)
    for k, v in BITSTREAMS.items():
        if len(sys.argv) > 1 and k not in sys.argv[1:]:
            continue
        save_bitstream(k, *v)
