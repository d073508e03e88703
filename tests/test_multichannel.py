"""Multichannel AAC-LC (channel configurations 3..7: SCE / CPE / LFE element lists,
SyntacticElements.process A/syntax/SyntacticElements.java:235-248 + SampleBuffer.accept's channel
interleave S/SampleBuffer.java:187-207): host parse round trips here, GPU decode against the
restatement (each element decoded as its own mono/stereo stream, channels interleaved in element
order) with -m gpu."""
import numpy as np
import pytest

from jaadec_amd import native as N
from oracle import oracle as O

IDS = N.MC_ELEMENTS


def mc_synth(cc: int, n_streams: int = 2, fps: int = 12, seed: int = 0, config: int = 3):
    """A multichannel batch from per-element synthetic batches (C3-style window switching + TNS;
    no PNS: the static LCG of a combined stream runs through all elements in parse order)."""
    els = []
    for k, i in enumerate(IDS[cc]):
        p = N.synth_params(config, n_streams=n_streams, frames_per_stream=fps, channel_config=2 if i == 1 else 1,
                           pns_percent=0)
        p.seed = p.seed + 0x100 * (k + 1) + seed
        if i == 3:
            p.window_switching = 0  # LFE: long windows (the parser accepts either)
        els.append(N.synth_batch(p))
    # every element's ch-frames start from the same (unused) LCG state
    return N.mc_batch(els, IDS[cc])


@pytest.mark.parametrize("cc", [3, 4, 5, 6, 7])
def test_element_layout(cc):
    cfg = N.make_cfg(channel_config=cc)
    assert N.core_channels(cfg) == {3: 3, 4: 4, 5: 5, 6: 6, 7: 8}[cc]
    b = mc_synth(cc)
    assert b.nch == N.core_channels(cfg) and b.ms_used.shape == (b.n_frames, 2 * N.n_cpe(cfg))


@pytest.mark.parametrize("cc", [3, 4, 5, 6, 7])
def test_write_parse_round_trip(cc):
    b = mc_synth(cc, n_streams=1, fps=10)
    frames = O.write_frames_mc(b, 3, IDS[cc])
    P = N.Parser(N.make_cfg(channel_config=cc))
    P.pns_state = int(b.ics["pns_state"][0])
    got = P.parse(frames)
    for k in ("q", "sf", "cb", "ics", "ms_used"):
        assert getattr(got, k).tobytes() == getattr(b, k).tobytes(), k


def test_parse_rejects_wrong_element_sequences():
    b = mc_synth(6, n_streams=1, fps=2)
    frames = O.write_frames_mc(b, 3, IDS[6])
    P = N.Parser(N.make_cfg(channel_config=5))  # 5.0 expects SCE CPE CPE, the frame adds an LFE
    with pytest.raises(N.JaadError) as e:
        P.parse(frames[:1])
    assert e.value.status == N.ERR_UNSUPPORTED
    short = mc_synth(5, n_streams=1, fps=2)
    frames5 = O.write_frames_mc(short, 3, IDS[5])
    P6 = N.Parser(N.make_cfg(channel_config=6))  # 5.1 without its LFE
    with pytest.raises(N.JaadError) as e:
        P6.parse(frames5[:1])
    assert e.value.status == N.ERR_UNSUPPORTED


def test_oracle_mc_matches_element_streams():
    """The multichannel oracle is the element decodes interleaved (structure check)."""
    b = mc_synth(3, n_streams=1, fps=6)
    got = O.decode_batch_mc(3, b, IDS[3], N.PCM_BIG_ENDIAN)
    assert got.shape == (6, 1024 * 3 * 2)
    s = got.view(">i2").reshape(6, 1024, 3)
    sce = N.Batch(b.q[0::3].copy(), b.sf[0::3].copy(), b.cb[0::3].copy(), b.ics[0::3].copy(), None,
                  b.tns[0::3].copy() if b.tns is not None else None, b.stream_slot.copy(), b.frame_begin.copy(), 1)
    mono = O.decode_batch(N.make_cfg(channel_config=1), sce, O.Streams(1), N.PCM_BIG_ENDIAN)
    assert (mono.view(">i2").reshape(6, 1024, 2)[:, :, 0] == s[:, :, 0]).all()


@pytest.mark.gpu
@pytest.mark.parametrize("cc", [3, 4, 5, 6, 7])
@pytest.mark.parametrize("flags", [N.PCM_BIG_ENDIAN, N.PCM_FLOAT32])
def test_gpu_decode_matches_oracle(cc, flags):
    b = mc_synth(cc, n_streams=3, fps=30)
    cfg = N.make_cfg(channel_config=cc)
    with N.Context(cfg, 3) as ctx:
        got = ctx.decode(b, flags)
    want = O.decode_batch_mc(3, b, IDS[cc], flags, threads=8)
    assert got.shape == want.shape
    assert (got == want).all(), np.flatnonzero(got.reshape(-1) != want.reshape(-1))[:8]


@pytest.mark.gpu
def test_gpu_continuation_and_state_roundtrip():
    b = mc_synth(6, n_streams=2, fps=24)
    cfg = N.make_cfg(channel_config=6)
    want = O.decode_batch_mc(3, b, IDS[6], N.PCM_BIG_ENDIAN)
    first, second = b.split_frames(10)
    with N.Context(cfg, 2) as ctx:
        g1 = ctx.decode(first)
        blob = ctx.state_export(1)
        g2 = ctx.decode(second)
        with N.Context(cfg, 2) as ctx2:  # stream 1 resumed in another context
            ctx2.state_import(1, blob)
            g2b = ctx2.decode(second.select_runs([1]))
    fb = b.frame_begin
    for r in range(2):
        assert (g1[10 * r:10 * (r + 1)] == want[fb[r]:fb[r] + 10]).all()
        assert (g2[14 * r:14 * (r + 1)] == want[fb[r] + 10:fb[r + 1]]).all()
    assert (g2b == want[fb[1] + 10:fb[2]]).all()


@pytest.mark.gpu
def test_gpu_bitstream_to_pcm_through_the_decoder_facade():
    """An ADTS 5.1 stream (channel_configuration 6) through ADTSDemultiplexer + Decoder.decodeFrame:
    6 interleaved channels per sample, equal to the restatement."""
    from jaadec_amd.decoder import ADTSDemultiplexer, Decoder, SampleBuffer
    b = mc_synth(6, n_streams=1, fps=8)
    frames = O.write_frames_mc(b, 3, IDS[6])
    demux = ADTSDemultiplexer(O.adts_wrap(frames, 3, 6))
    dec = Decoder.create(demux.getDecoderInfo())
    dec._parse([])
    dec._parser.pns_state = int(b.ics["pns_state"][0])
    want = O.decode_batch_mc(3, b, IDS[6], N.PCM_BIG_ENDIAN)
    for i in range(8):
        buf = SampleBuffer()
        dec.decodeFrame(demux.readNextFrame(), buf)
        assert buf.getData() == want[i].tobytes(), i
        assert buf.getChannels() == 6
    assert dec.getConfig().getChannelCount() == 6
    dec.close()


def _pce_asc(sfi: int, front, side=(), back=(), n_lfe: int = 0, pce_sfi: int | None = None, aot: int = 2) -> bytes:
    """An AudioSpecificConfig with channelConfiguration 0 and its program_config_element
    (PCE.read / decode, A/syntax/PCE.java:47-52,133-188): element lists as is_cpe flags."""
    bits = f"{aot:05b}{sfi:04b}{0:04b}000"                           # GASpecificConfig
    bits += f"{0:04b}{1:02b}{(sfi if pce_sfi is None else pce_sfi):04b}"  # tag, LC, rate
    bits += f"{len(front):04b}{len(side):04b}{len(back):04b}{n_lfe:02b}{0:03b}{0:04b}000"
    for lst in (front, side, back):
        for k, cpe in enumerate(lst):
            bits += f"{int(cpe):01b}{k:04b}"
    bits += "".join(f"{k:04b}" for k in range(n_lfe))
    bits += "0" * (-len(bits) % 8) + f"{0:08b}"                      # byte_align, no comment
    bits += "0" * (-len(bits) % 8)
    return int(bits, 2).to_bytes(len(bits) // 8, "big")


@pytest.mark.parametrize("layout, cc", [
    (dict(front=[True]), 2),                                          # stereo
    (dict(front=[False]), 1),                                         # mono
    (dict(front=[False, True], back=[True], n_lfe=1), 6),             # 5.1
    (dict(front=[False, True], side=[True], n_lfe=1), 6),             # 5.1, surrounds as side elements
    (dict(front=[False, True], back=[False]), 4),                     # 4.0: C, L/R, back centre
    (dict(front=[False, True], n_lfe=1), 4),                          # 3.1 counts 4 channels -> 4.0 list
    (dict(front=[False, True, True], back=[True], n_lfe=1), 7),       # 8 channels -> 7.1
])
def test_asc_program_config_element_layouts(layout, cc):
    """DecoderConfig.decode with channelConfiguration 0 (A/DecoderConfig.java:231-235): the PCE's
    channel count picks the configuration (PCE.getChannelConfiguration -> forChannelCount)."""
    cfg = N.asc_parse(_pce_asc(3, **layout))
    assert (cfg.channel_config, cfg.sf_index, cfg.profile) == (cc, 3, 2)


def test_asc_program_config_element_rate_and_refusals():
    # setAudioDecoderInfo(pce) replaces sampleFrequency with the PCE's rate after outputFrequency was
    # set to the ASC's (A/DecoderConfig.java:180, 231-235): with different rates the reference's
    # getSampleLength becomes 2048 at the ASC's output rate -- not reproduced, refused
    with pytest.raises(N.JaadError) as e:
        N.asc_parse(_pce_asc(4, front=[True], pce_sfi=3))
    assert e.value.status == N.ERR_UNSUPPORTED
    assert N.asc_parse(_pce_asc(3, front=[True], pce_sfi=3)).sf_index == 3  # equal rates decode
    for layout in (dict(front=[False, False]),                        # dual mono: SCE SCE is not the CPE list
                   dict(front=[True, False]),                         # CPE then SCE: not the 3.0 list
                   dict(front=[False, True, True], back=[True]),      # 7 channels: forChannelCount throws
                   dict(front=[], n_lfe=1)):                          # a lone LFE
        with pytest.raises(N.JaadError) as e:
            N.asc_parse(_pce_asc(3, **layout))
        assert e.value.status == N.ERR_UNSUPPORTED, layout


@pytest.mark.gpu
def test_gpu_pce_config_decodes_like_the_standard_configuration():
    """A 5.1 stream whose AudioSpecificConfig carries a PCE (as an MP4 DSI can) through
    Decoder.create(asc) + decodeFrame: the PCM of channel configuration 6."""
    from jaadec_amd.decoder import Decoder, SampleBuffer
    b = mc_synth(6, n_streams=1, fps=6)
    frames = O.write_frames_mc(b, 3, IDS[6])
    dec = Decoder.create(_pce_asc(3, front=[False, True], back=[True], n_lfe=1))
    assert dec.getConfig().getChannelCount() == 6
    dec._parse([])
    dec._parser.pns_state = int(b.ics["pns_state"][0])
    want = O.decode_batch_mc(3, b, IDS[6], N.PCM_BIG_ENDIAN)
    for i in range(6):
        buf = SampleBuffer()
        dec.decodeFrame(frames[i], buf)
        assert buf.getData() == want[i].tobytes(), i
    dec.close()


def _pce_element(sfi: int, front, side=(), back=(), n_lfe: int = 0) -> bytes:
    """A program_config_element as the first element of a raw_data_block (id 5, tag, PCE.decode);
    it ends byte-aligned, so it is prepended to a frame's bytes."""
    bits = f"{5:03b}{0:04b}{1:02b}{sfi:04b}"
    bits += f"{len(front):04b}{len(side):04b}{len(back):04b}{n_lfe:02b}{0:03b}{0:04b}000"
    for lst in (front, side, back):
        for k, cpe in enumerate(lst):
            bits += f"{int(cpe):01b}{k:04b}"
    bits += "".join(f"{k:04b}" for k in range(n_lfe))
    bits += "0" * (-len(bits) % 8) + f"{0:08b}"
    return int(bits, 2).to_bytes(len(bits) // 8, "big")


def test_raw_pce_cfg():
    raw = _pce_element(3, front=[False, True], back=[True], n_lfe=1) + b"\xe0"  # PCE, END
    cfg = N.raw_pce_cfg(raw)
    assert (cfg.channel_config, cfg.sf_index) == (6, 3)
    with pytest.raises(N.JaadError) as e:
        N.raw_pce_cfg(b"\xe0")  # END: no PCE first
    assert e.value.status == N.ERR_BITSTREAM
    assert N.adts_cfg(N.adts_frames(O.adts_wrap([raw], 3, 0)).__next__()[0]).channel_config == 0


@pytest.mark.gpu
def test_gpu_adts_channel_config_0_takes_the_layout_from_the_frames_pce():
    """ADTS channel_configuration 0: the first frame's PCE sets the configuration
    (SyntacticElements.decode -> setAudioDecoderInfo, A/syntax/SyntacticElements.java:153-156);
    later PCEs are skipped as elements.  PCM equal to the channel configuration 6 decode."""
    from jaadec_amd.decoder import ADTSDemultiplexer, Decoder, SampleBuffer
    b = mc_synth(6, n_streams=1, fps=6)
    frames = O.write_frames_mc(b, 3, IDS[6])
    pce = _pce_element(3, front=[False, True], back=[True], n_lfe=1)
    frames = [pce + f if i in (0, 3) else f for i, f in enumerate(frames)]
    demux = ADTSDemultiplexer(O.adts_wrap(frames, 3, 0))
    dec = Decoder.create(demux.getDecoderInfo())
    assert dec.getConfig().getChannelCount() == 0
    want = O.decode_batch_mc(3, b, IDS[6], N.PCM_BIG_ENDIAN)
    for i in range(6):
        buf = SampleBuffer()
        dec.decodeFrame(demux.readNextFrame(), buf)
        assert buf.getData() == want[i].tobytes(), i
    assert dec.getConfig().getChannelCount() == 6
    dec.close()
