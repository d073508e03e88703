"""The host mirror of the reference interface (A/Decoder.java, A/DecoderConfig.java, S/SampleBuffer.java)."""
import numpy as np
import pytest

from jaadec_amd import native as N
from jaadec_amd.decoder import AACException, Decoder, DecoderConfig, SampleBuffer


@pytest.mark.parametrize("asc,aot,sfi,ch", [
    (bytes([0x12, 0x08]), 2, 4, 1),   # C1: LC, 44.1 kHz, mono
    (bytes([0x11, 0x90]), 2, 3, 2),   # LC, 48 kHz, stereo
    (bytes([0x11, 0x88]), 2, 3, 1),
])
def test_audio_specific_config(asc, aot, sfi, ch):
    c = DecoderConfig.decode(asc)
    assert (c.profile, c.sf_index, c.channel_config) == (aot, sfi, ch)
    assert c.getSampleLength() == 1024
    assert c.getChannelCount() == 2  # mono is upmixed (A/DecoderConfig.java:108-115)
    assert c.getSampleFrequency() == [96000, 88200, 64000, 48000, 44100][sfi]


def test_explicit_frequency_maps_to_nearest_index():
    # AOT 2, sfi 15, 24-bit frequency 44100, ch 2, then GASpecificConfig zeros
    bits = f"{2:05b}{15:04b}{44100:024b}{2:04b}000"
    bits += "0" * (-len(bits) % 8)
    asc = int(bits, 2).to_bytes(len(bits) // 8, "big")
    assert DecoderConfig.decode(asc).sf_index == 4


def test_explicit_sbr_and_ps_configs():
    c = DecoderConfig.decode(bytes([0x2B, 0x11, 0x88, 0x00]))  # AOT 5, 24 kHz core -> 48 kHz, stereo
    assert (c.sbr, c.ps, c.sf_index, c.ext_sf_index, c.getSampleLength(), c.getOutputFrequency()) == \
        (True, False, 6, 3, 2048, 48000)
    c = DecoderConfig.decode(bytes([0xEB, 0x09, 0x88, 0x00]))  # AOT 29: mono core + SBR + PS
    assert (c.sbr, c.ps, c.channel_config, c.getChannelCount()) == (True, True, 1, 2)


@pytest.mark.parametrize("asc,msg", [
    (bytes([0x0A, 0x10]), "profile"),               # AOT 1 (Main): ICPrediction out of scope
    (bytes([0x12, 0x0C]), "960"),                   # frameLengthFlag
    (bytes([0x12]), "end"),
])
def test_unsupported_or_truncated_config_raises(asc, msg):
    with pytest.raises(AACException, match=msg):
        DecoderConfig.decode(asc)


def test_samplebuffer_default_big_endian_and_swap():
    b = SampleBuffer()
    assert b.isBigEndian()
    b._set(bytes([0x12, 0x34, 0xAB, 0xCD]), 48000)
    b.setBigEndian(False)
    assert b.getData() == bytes([0x34, 0x12, 0xCD, 0xAB]) and not b.isBigEndian()
    b.setBigEndian(False)  # no change
    assert b.getData() == bytes([0x34, 0x12, 0xCD, 0xAB])


def test_decoder_create_without_gpu_raises_aacexception():
    from conftest import gpu_available
    if gpu_available():
        pytest.skip("a GPU is present")
    with pytest.raises(AACException, match="device"):
        Decoder.create(bytes([0x11, 0x90]))


@pytest.mark.gpu
@pytest.mark.parametrize("big_endian", [True, False])
def test_decode_frames_matches_oracle(big_endian):
    from oracle import oracle as O
    full = N.synth_batch(N.synth_params(3, n_streams=1, frames_per_stream=14))
    batch, tail = full.split_frames(10)
    dec = Decoder.create(bytes([0x11, 0x90]))
    bufs = [SampleBuffer(big_endian) for _ in range(batch.n_frames)]
    dec.decodeFrames(batch, bufs)
    flags = N.PCM_BIG_ENDIAN if big_endian else N.PCM_LITTLE_ENDIAN
    want_full = O.decode_batch(N.make_cfg(), full, O.Streams(1), flags)
    for i, b in enumerate(bufs):
        assert b.getData() == want_full[i].tobytes()
        assert (b.sample_rate, b.channels, b.bits_per_sample) == (48000, 2, 16)
    # frame-at-a-time decodeFrame continues the same stream state
    for k in range(4):
        one, tail = tail.split_frames(1)
        buf = SampleBuffer(big_endian)
        dec.decodeFrame(one, buf)
        assert buf.getData() == want_full[10 + k].tobytes()
    dec.close()


@pytest.mark.gpu
def test_mixed_endianness_buffers():
    from oracle import oracle as O
    batch = N.synth_batch(N.synth_params(2, n_streams=1, frames_per_stream=4))
    dec = Decoder.create(bytes([0x11, 0x90]))
    bufs = [SampleBuffer(i % 2 == 0) for i in range(4)]
    dec.decodeFrames(batch, bufs)
    be = O.decode_batch(N.make_cfg(), batch, O.Streams(1), N.PCM_BIG_ENDIAN)
    le = O.decode_batch(N.make_cfg(), batch, O.Streams(1), N.PCM_LITTLE_ENDIAN)
    for i, b in enumerate(bufs):
        assert b.getData() == (be if i % 2 == 0 else le)[i].tobytes()
    dec.close()


def test_adts_demultiplexer_mirror():
    from jaadec_amd.decoder import ADTSDemultiplexer
    from oracle import oracle as O
    p = N.synth_params(2, n_streams=1, frames_per_stream=3)
    b = N.synth_batch(p)
    frames = O.write_frames(b, p.sf_index)
    demux = ADTSDemultiplexer(O.adts_wrap(frames, p.sf_index, p.channel_config))
    assert (demux.getSampleFrequency(), demux.getChannelCount()) == (48000, 2)
    assert demux.getDecoderInfo().cfg().sf_index == 3
    got = [demux.readNextFrame() for _ in range(3)]
    assert got == frames
    with pytest.raises(EOFError):
        demux.readNextFrame()
    with pytest.raises(OSError):
        ADTSDemultiplexer(bytes(100))


@pytest.mark.gpu
def test_decode_raw_frames_from_adts_matches_oracle():
    """Main.decodeAAC's loop (S/Main.java:82-111): ADTS -> decodeFrame(raw bytes) -> SampleBuffer."""
    from jaadec_amd.decoder import ADTSDemultiplexer
    from oracle import oracle as O
    p = N.synth_params(3, n_streams=1, frames_per_stream=12)
    b = N.synth_batch(p)
    demux = ADTSDemultiplexer(O.adts_wrap(O.write_frames(b, p.sf_index), p.sf_index, p.channel_config))
    dec = Decoder.create(demux.getDecoderInfo())
    dec._parse([])  # parser up front so the PNS LCG can be seeded like the synthetic batch's
    dec._parser.pns_state = int(b.ics["pns_state"][0])
    want = O.decode_batch(N.make_cfg(), b, O.Streams(1), N.PCM_BIG_ENDIAN)
    for i in range(12):
        buf = SampleBuffer()
        dec.decodeFrame(demux.readNextFrame(), buf)
        assert buf.getData() == want[i].tobytes()
    dec.close()


@pytest.mark.gpu
def test_truncated_frame_is_dropped_and_the_buffer_keeps_the_last_pcm():
    """A/Decoder.java:89-101: decodeFrame swallows an EOSException (warning), the Receiver is not
    called, the frame still counts; decode0 lets it propagate."""
    from jaadec_amd.decoder import EOSException
    from oracle import oracle as O
    p = N.synth_params(2, n_streams=1, frames_per_stream=4)
    b = N.synth_batch(p)
    frames = O.write_frames(b, p.sf_index)
    want = O.decode_batch(N.make_cfg(), b, O.Streams(1), N.PCM_BIG_ENDIAN)
    dec = Decoder.create(DecoderConfig.decode(bytes([0x11, 0x90])))
    buf = SampleBuffer()
    dec.decodeFrame(frames[0], buf)
    assert buf.getData() == want[0].tobytes()
    dec.decodeFrame(frames[1][:len(frames[1]) // 2], buf)
    assert buf.getData() == want[0].tobytes() and dec.frames == 2
    with pytest.raises(EOSException):
        dec.decode0(frames[1][:10], buf)
    # the dropped frame changed nothing: frame 1 decodes as if it came right after frame 0
    dec.decodeFrame(frames[1], buf)
    assert buf.getData() == want[1].tobytes()
    fmt = dec.getAudioFormat()
    assert (fmt.sample_rate, fmt.bits, fmt.channels, fmt.big_endian) == (48000, 16, 2, False)
    dec.close()


@pytest.mark.gpu
def test_rejected_batch_rolls_the_parser_back():
    """decodeFrames parses the whole list before the DSP runs: when the batch is then rejected,
    the parser state (PNS LCG, window shapes) is rolled back, so the frames decode afterwards
    exactly as if the failed call had never happened."""
    from oracle import oracle as O
    p = N.synth_params(3, n_streams=1, frames_per_stream=8, pns_percent=10)
    b = N.synth_batch(p)
    frames = O.write_frames(b, p.sf_index)
    want = O.decode_batch(N.make_cfg(), b, O.Streams(1), N.PCM_BIG_ENDIAN)
    dec = Decoder.create(bytes([0x11, 0x90]))
    dec._parse([])
    dec._parser.pns_state = int(b.ics["pns_state"][0])
    bufs = [SampleBuffer() for _ in range(3)]
    dec.decodeFrames(frames[:3], bufs)
    with pytest.raises(AACException):
        dec.decodeFrames(frames[3:6], bufs[:2])  # parsed, then rejected (buffer count)
    bufs = [SampleBuffer() for _ in range(5)]
    dec.decodeFrames(frames[3:], bufs)
    for i, buf in enumerate(bufs):
        assert buf.getData() == want[3 + i].tobytes(), i
    dec.close()


def _asc(bits: str) -> bytes:
    bits += "0" * (-len(bits) % 8)
    return int(bits, 2).to_bytes(len(bits) // 8, "big")


def test_sync_extension_signals_sbr_and_asc_keeps_the_core_rate():
    """readSyncExtension (A/DecoderConfig.java:260-291): an AOT 2 config carrying 0x2B7 + AAC_SBR
    + sbrPresent is explicit SBR at the signalled rate (0x548: psPresent).  Without it the config
    keeps outputFrequency = the core rate (:180): implicit SBR found later runs downsampled for an
    ASC-created decoder, doubled for an ADTS-created one (AudioDecoderInfo, setSBRPresent :124-135)."""
    core = f"{2:05b}{6:04b}{2:04b}000"                     # LC, 24 kHz, stereo, GASpecificConfig
    c = DecoderConfig.decode(_asc(core + f"{0x2B7:011b}{5:05b}1{3:04b}"))
    assert (c.sbr, c.ext_sf_index, c.getSampleLength(), c.getOutputFrequency()) == (True, 3, 2048, 48000)
    c = DecoderConfig.decode(_asc(f"{2:05b}{6:04b}{1:04b}000" + f"{0x2B7:011b}{5:05b}1{3:04b}{0x548:011b}1"))
    assert (c.sbr, c.ps, c.channel_config, c.ext_sf_index) == (True, True, 1, 3)
    c = DecoderConfig.decode(_asc(core + f"{0x2B7:011b}{5:05b}0"))  # sbrPresent = 0
    assert (c.sbr, c.from_asc, c.getSampleLength()) == (False, True, 1024)
    plain = DecoderConfig.decode(_asc(core))
    assert not plain.sbr and plain.from_asc
    up_asc = N.implicit_sbr_cfg(plain.cfg(), from_asc=True)
    up_adts = N.implicit_sbr_cfg(plain.cfg())
    assert (up_asc.ext_sf_index, up_adts.ext_sf_index) == (6, 3)


@pytest.mark.gpu
@pytest.mark.parametrize("via", ["asc", "adts"])
def test_implicit_sbr_rate_follows_the_creation_path(via):
    """Main.decodeMP4 (S/Main.java:62, Decoder.create(DSI)) vs Main.decodeAAC (:84, ADTS header):
    the same AOT 2 frames with SBR in FIL elements decode to 1024 core-rate samples through an
    ASC-created decoder (SynthesisFilterbank32) and to 2048 doubled-rate samples through an
    ADTS-created one, each equal to the restatement."""
    from jaadec_amd.decoder import ADTSDemultiplexer
    from oracle import oracle as O
    p = N.synth_params(4, n_streams=1, frames_per_stream=10)
    b = N.synth_batch(p)
    # the SBR frequency tables follow the SBR output rate (SBR.sample_rate = outputFrequency,
    # A/sbr/SBR.java:102): the core rate through the ASC, twice it through ADTS
    out_sf = p.sf_index if via == "asc" else p.sf_index - 3
    frames = O.write_frames(b, p.sf_index, sbr_writer=O.SbrWriter(out_sf, 5))
    if via == "asc":
        dec = Decoder.create(_asc(f"{2:05b}{p.sf_index:04b}{2:04b}000"))
        cfg = N.make_cfg(p.sf_index, 2, sbr=True, down=True)
        frames_in = frames
    else:
        demux = ADTSDemultiplexer(O.adts_wrap(frames, p.sf_index, 2))
        dec = Decoder.create(demux.getDecoderInfo())
        cfg = N.cfg_for(p)
        frames_in = [demux.readNextFrame() for _ in range(10)]
    want = O.decode_batch(cfg, b, O.Streams(1), N.PCM_BIG_ENDIAN)
    for i in range(10):
        buf = SampleBuffer()
        dec.decodeFrame(frames_in[i], buf)
        assert buf.getData() == want[i].tobytes(), i
    c = dec.getConfig()
    assert c.getSampleLength() == (1024 if via == "asc" else 2048)
    assert buf.getSampleRate() == (24000 if via == "asc" else 48000)
    dec.close()
