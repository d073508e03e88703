// MP4 transport feeder (include/jaad_mp4.h): the box walk and sample table of the reference's MP4
// API restated for a file image in memory (M/ = mp4/src/main/java/net/sourceforge/jaad/mp4/).
//   box header (size, 'uuid', 64-bit size, size 0 = to the end)   M/boxes/BoxFactory.java
//   moov -> trak -> mdia (mdhd, hdlr) -> minf -> stbl               M/api/Movie.java:15-62, Track.java:44-88
//   stsd -> mp4a (AudioSampleEntry) -> esds descriptors             M/api/AudioTrack.java:46-77,
//                                                                   M/boxes/impl/sampleentries/*.java,
//                                                                   M/od/Descriptor.java, ESDescriptor.java,
//                                                                   DecoderConfigDescriptor.java
//   stsz/stz2, stco/co64, stsc, stts -> frames sorted by time       M/api/Track.java:90-155
#include "../../include/jaad_mp4.h"

#include <algorithm>
#include <cstring>
#include <new>
#include <vector>

namespace {

constexpr uint32_t fourcc(const char (&s)[5])
{
    return (uint32_t)(uint8_t)s[0] << 24 | (uint32_t)(uint8_t)s[1] << 16 | (uint32_t)(uint8_t)s[2] << 8 | (uint8_t)s[3];
}

struct Span {
    const uint8_t* p = nullptr;
    size_t n = 0;
};

struct Box {
    uint32_t type = 0;
    Span body;               // after the header (and after a 'uuid' user type)
    bool truncated = false;  // top level only: the image ends inside this box
};

// big-endian reader over a span; any read past the end sets bad
struct Rd {
    Span s;
    size_t pos = 0;
    bool bad = false;
    uint64_t u(int bytes)
    {
        if (pos + (size_t)bytes > s.n) {
            bad = true;
            pos = s.n;
            return 0;
        }
        uint64_t v = 0;
        for (int i = 0; i < bytes; i++) v = v << 8 | s.p[pos++];
        return v;
    }
    void skip(size_t k)
    {
        if (pos + k > s.n) {
            bad = true;
            pos = s.n;
        } else {
            pos += k;
        }
    }
    size_t left() const { return s.n - pos; }
};

// the boxes directly inside a span (BoxFactory.parseBox: 32-bit size, 1 = 64-bit size, 0 = rest)
// top_level: a last box that runs past the end of the image is kept, clipped and marked (a file
// cut inside mdat still has its moov; the reference skips mdat without reading it)
int children(Span s, std::vector<Box>& out, bool top_level = false)
{
    out.clear();
    size_t pos = 0;
    while (pos + 8 <= s.n) {
        Rd r{Span{s.p + pos, s.n - pos}};
        uint64_t size = r.u(4);
        const uint32_t type = (uint32_t)r.u(4);
        size_t hdr = 8;
        if (size == 1) {
            size = r.u(8);
            hdr = 16;
            if (r.bad) return JAAD_ERR_EOS;
        } else if (size == 0) {
            size = s.n - pos;
        }
        if (size < hdr) return JAAD_ERR_BITSTREAM;
        bool cut = false;
        if (size > s.n - pos) {
            if (!top_level) return JAAD_ERR_EOS;
            size = s.n - pos;
            cut = true;
        }
        if (type == fourcc("uuid")) hdr += 16;
        if (hdr > size) return cut ? JAAD_ERR_EOS : JAAD_ERR_BITSTREAM;
        out.push_back(Box{type, Span{s.p + pos + hdr, (size_t)size - hdr}, cut});
        pos += (size_t)size;
    }
    return JAAD_OK;
}

const Box* find(const std::vector<Box>& v, uint32_t type)
{
    for (const Box& b : v)
        if (b.type == type) return &b;
    return nullptr;
}

// one descriptor (Descriptor.createDescriptor): tag, 7-bit-continued size, body
struct Desc {
    int tag = 0;
    Span body;
};
bool read_desc(Rd& r, Desc& d)
{
    d.tag = (int)r.u(1);
    uint32_t size = 0;
    int b;
    int n = 0;
    do {
        b = (int)r.u(1);
        size = size << 7 | (uint32_t)(b & 0x7F);
    } while ((b & 0x80) && ++n < 4 && !r.bad);
    if (r.bad || size > r.left()) return false;
    d.body = Span{r.s.p + r.pos, size};
    r.skip(size);
    return true;
}

struct Frame {
    uint64_t offset;
    uint32_t size;
    double time;
};

struct Track {
    jaad_mp4_track info{};
    std::vector<uint8_t> dsi;
    std::vector<Frame> frames;
};

// ESDBox -> ES_Descriptor -> (children -> their DecoderSpecificInfo children), Track.java:158-173
int parse_esds(Span esds, std::vector<uint8_t>& dsi)
{
    Rd r{esds};
    r.skip(4);  // full box version/flags
    Desc es;
    if (!read_desc(r, es)) return JAAD_ERR_EOS;
    if (es.tag != 3) return JAAD_OK;  // not an ES_Descriptor: no DecoderSpecificInfo found
    Rd e{es.body};
    e.skip(2);  // ES_ID
    const int flags = (int)e.u(1);
    if (flags & 0x80) e.skip(2);           // dependsOn_ES_ID
    if (flags & 0x40) e.skip(e.u(1));      // URL; the OCR flag is not read (ESDescriptor.java:decode)
    while (!e.bad && e.left() > 0) {
        Desc c;
        if (!read_desc(e, c)) return JAAD_ERR_EOS;
        if (c.tag != 4) continue;  // only DecoderConfigDescriptor has parsed children here
        Rd cr{c.body};
        cr.skip(13);               // objectProfile, streamType, bufferSize, max/avg bitrate
        while (!cr.bad && cr.left() > 0) {
            Desc g;
            if (!read_desc(cr, g)) return JAAD_ERR_EOS;
            if (g.tag == 5) dsi.assign(g.body.p, g.body.p + g.body.n);
        }
    }
    return e.bad ? JAAD_ERR_EOS : JAAD_OK;
}

int parse_trak(Span trak, std::vector<Track>& tracks, size_t file_bytes)
{
    std::vector<Box> tk, md, mi, st, sd;
    int rc;
    if ((rc = children(trak, tk))) return rc;
    const Box* tkhd = find(tk, fourcc("tkhd"));
    const Box* mdia = find(tk, fourcc("mdia"));
    if (!mdia) return JAAD_ERR_BITSTREAM;
    if ((rc = children(mdia->body, md))) return rc;
    const Box* hdlr = find(md, fourcc("hdlr"));
    const Box* mdhd = find(md, fourcc("mdhd"));
    const Box* minf = find(md, fourcc("minf"));
    if (!hdlr || !mdhd || !minf) return JAAD_ERR_BITSTREAM;
    Rd h{hdlr->body};
    h.skip(8);  // version/flags, pre_defined
    if ((uint32_t)h.u(4) != fourcc("soun") || h.bad) return JAAD_OK;  // Movie.createTrack: audio only here
    Track T;
    if (tkhd) {
        Rd t{tkhd->body};
        const int ver = (int)t.u(1);
        t.skip(3 + (ver == 1 ? 16 : 8));
        T.info.track_id = (uint32_t)t.u(4);
    }
    {
        Rd m{mdhd->body};
        const int ver = (int)m.u(1);
        m.skip(3 + (ver == 1 ? 16 : 8));
        T.info.timescale = (uint32_t)m.u(4);
        if (m.bad) return JAAD_ERR_EOS;
    }
    if ((rc = children(minf->body, mi))) return rc;
    const Box* stbl = find(mi, fourcc("stbl"));
    if (!stbl) return JAAD_ERR_BITSTREAM;
    if ((rc = children(stbl->body, st))) return rc;
    // sample description: the first entry (AudioTrack.java:55-57)
    if (const Box* stsd = find(st, fourcc("stsd"))) {
        Rd s{stsd->body};
        s.skip(8);  // version/flags, entry_count
        if ((rc = children(Span{stsd->body.p + s.pos, s.left()}, sd))) return rc;
        if (!sd.empty()) {
            const Box& e = sd[0];
            T.info.sample_entry = e.type;
            Rd a{e.body};
            a.skip(8);   // SampleEntry: reserved, data_reference_index
            a.skip(8);   // AudioSampleEntry: reserved
            T.info.channel_count = (uint32_t)a.u(2);
            T.info.sample_size = (uint32_t)a.u(2);
            a.skip(4);
            T.info.sample_rate = (uint32_t)a.u(2);
            a.skip(2);
            if (a.bad) return JAAD_ERR_EOS;
            std::vector<Box> ec;
            if ((rc = children(Span{e.body.p + a.pos, a.left()}, ec))) return rc;
            if (const Box* esds = find(ec, fourcc("esds")))
                if ((rc = parse_esds(esds->body, T.dsi))) return rc;
            T.info.dsi_bytes = (uint32_t)T.dsi.size();
        }
    }
    // sample table (Track.parseSampleTable)
    const Box* stsz = find(st, fourcc("stsz"));
    const Box* stz2 = find(st, fourcc("stz2"));
    const Box* stco = find(st, fourcc("stco"));
    const Box* co64 = find(st, fourcc("co64"));
    const Box* stsc = find(st, fourcc("stsc"));
    const Box* stts = find(st, fourcc("stts"));
    if ((!stsz && !stz2) || (!stco && !co64) || !stsc || !stts) {
        if (st.empty()) {  // an empty stbl has no frames (Track.java:81-86)
            tracks.push_back(std::move(T));
            return JAAD_OK;
        }
        return JAAD_ERR_BITSTREAM;
    }
    std::vector<uint32_t> sizes;
    {
        Rd z{(stsz ? stsz : stz2)->body};
        z.skip(4);
        int field = 32;
        uint32_t fixed = 0;
        if (stsz) {
            fixed = (uint32_t)z.u(4);
        } else {
            z.skip(3);
            field = (int)z.u(1);
        }
        const uint64_t count = z.u(4);
        if (z.bad) return JAAD_ERR_EOS;
        if (count > (1u << 28)) return JAAD_ERR_BITSTREAM;
        // every sample is bytes of this file: a count the file cannot hold is corrupt (and would
        // size the tables below from a ~100-byte file)
        if (stsz && fixed) {
            if (count > file_bytes / fixed) return JAAD_ERR_BITSTREAM;
        } else if (count > z.left() * (field == 4 ? 2 : 1)) {
            return JAAD_ERR_EOS;
        }
        sizes.resize((size_t)count);
        if (stsz && fixed) {
            std::fill(sizes.begin(), sizes.end(), fixed);
        } else if (field == 4) {
            for (size_t i = 0; i < count; i += 2) {
                const int x = (int)z.u(1);
                sizes[i] = (uint32_t)(x >> 4 & 0xF);
                if (i + 1 < count) sizes[i + 1] = (uint32_t)(x & 0xF);
            }
        } else {
            const int b = field / 8;
            if (b != 1 && b != 2 && b != 4) return JAAD_ERR_BITSTREAM;
            for (size_t i = 0; i < count; i++) sizes[i] = (uint32_t)z.u(b);
        }
        if (z.bad) return JAAD_ERR_EOS;
    }
    std::vector<uint64_t> chunks;
    {
        Rd c{(stco ? stco : co64)->body};
        c.skip(4);
        const uint64_t n = c.u(4);
        if (n > c.left()) return JAAD_ERR_EOS;
        chunks.resize((size_t)n);
        for (auto& o : chunks) o = c.u(stco ? 4 : 8);
        if (c.bad) return JAAD_ERR_EOS;
    }
    std::vector<uint64_t> first, per;
    {
        Rd c{stsc->body};
        c.skip(4);
        const uint64_t n = c.u(4);
        if (n > c.left()) return JAAD_ERR_EOS;
        for (uint64_t i = 0; i < n; i++) {
            first.push_back(c.u(4));
            per.push_back(c.u(4));
            c.skip(4);
        }
        if (c.bad) return JAAD_ERR_EOS;
    }
    std::vector<uint64_t> times(sizes.size(), 0);
    {
        Rd c{stts->body};
        c.skip(4);
        const uint64_t n = c.u(4);
        if (n > c.left()) return JAAD_ERR_EOS;
        uint64_t t = 0;
        size_t off = 0;
        for (uint64_t i = 0; i < n; i++) {
            const uint64_t cnt = c.u(4), delta = c.u(4);
            for (uint64_t j = 0; j < cnt; j++) {
                if (off + j >= times.size()) return JAAD_ERR_BITSTREAM;  // timeOffsets overflow in the reference
                times[off + j] = t;
                t += delta;
            }
            off += (size_t)cnt;
        }
        if (c.bad) return JAAD_ERR_EOS;
    }
    const double ts = (double)T.info.timescale;
    size_t cur = 0;
    for (size_t i = 0; i < first.size(); i++) {
        const uint64_t last = i + 1 < first.size() ? first[i + 1] - 1 : chunks.size();
        if (first[i] < 1) return JAAD_ERR_BITSTREAM;
        for (uint64_t j = first[i] - 1; j < last; j++) {
            if (j >= chunks.size()) return JAAD_ERR_BITSTREAM;
            uint64_t off = chunks[(size_t)j];
            for (uint64_t k = 0; k < per[i]; k++) {
                if (cur >= sizes.size()) return JAAD_ERR_BITSTREAM;
                T.frames.push_back(Frame{off, sizes[cur], (double)times[cur] / ts});
                off += sizes[cur];
                cur++;
            }
        }
    }
    // Collections.sort(frames) by time stamp; a stable sort keeps equal times in table order
    std::stable_sort(T.frames.begin(), T.frames.end(), [](const Frame& a, const Frame& b) { return a.time < b.time; });
    T.info.n_frames = (uint32_t)T.frames.size();
    tracks.push_back(std::move(T));
    return JAAD_OK;
}

}  // namespace

struct jaad_mp4 {
    std::vector<Track> tracks;
};

extern "C" {

static int mp4_open(const uint8_t* file, size_t bytes, jaad_mp4** out);

int jaad_mp4_open(const uint8_t* file, size_t bytes, jaad_mp4** out)
{
    if (!out || (!file && bytes)) return JAAD_ERR_INVALID_ARG;
    *out = nullptr;
    try {  // no C++ exception may cross the C ABI (a JVM / Python host would abort)
        return mp4_open(file, bytes, out);
    } catch (const std::bad_alloc&) {
        return JAAD_ERR_NOMEM;
    } catch (...) {
        return JAAD_ERR_BITSTREAM;
    }
}

static int mp4_open(const uint8_t* file, size_t bytes, jaad_mp4** out)
{
    std::vector<Box> top, moov;
    int rc = children(Span{file, bytes}, top, true);
    if (rc) return rc;
    const Box* mv = find(top, fourcc("moov"));
    if (!mv) return JAAD_ERR_BITSTREAM;
    if (mv->truncated) return JAAD_ERR_EOS;
    if ((rc = children(mv->body, moov))) return rc;
    jaad_mp4* m = new (std::nothrow) jaad_mp4;
    if (!m) return JAAD_ERR_NOMEM;
    for (const Box& b : moov) {
        if (b.type != fourcc("trak")) continue;
        if ((rc = parse_trak(b.body, m->tracks, bytes))) {
            delete m;
            return rc;
        }
    }
    *out = m;
    return JAAD_OK;
}

void jaad_mp4_close(jaad_mp4* m) { delete m; }

int jaad_mp4_track_count(const jaad_mp4* m) { return m ? (int)m->tracks.size() : 0; }

int jaad_mp4_track_info(const jaad_mp4* m, int track, jaad_mp4_track* info)
{
    if (!m || !info || track < 0 || track >= (int)m->tracks.size()) return JAAD_ERR_INVALID_ARG;
    *info = m->tracks[(size_t)track].info;
    return JAAD_OK;
}

int jaad_mp4_decoder_specific_info(const jaad_mp4* m, int track, const uint8_t** dsi, size_t* bytes)
{
    if (!m || !dsi || !bytes || track < 0 || track >= (int)m->tracks.size()) return JAAD_ERR_INVALID_ARG;
    const Track& T = m->tracks[(size_t)track];
    *dsi = T.dsi.empty() ? nullptr : T.dsi.data();
    *bytes = T.dsi.size();
    return JAAD_OK;
}

int jaad_mp4_frame(const jaad_mp4* m, int track, uint32_t i, uint64_t* offset, uint32_t* size, double* time)
{
    if (!m || track < 0 || track >= (int)m->tracks.size()) return JAAD_ERR_INVALID_ARG;
    const Track& T = m->tracks[(size_t)track];
    if (i >= T.frames.size()) return JAAD_ERR_EOS;
    if (offset) *offset = T.frames[i].offset;
    if (size) *size = T.frames[i].size;
    if (time) *time = T.frames[i].time;
    return JAAD_OK;
}

}  // extern "C"
