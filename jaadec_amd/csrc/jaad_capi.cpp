// C-ABI implementation (include/jaad_gpu.h): contexts, per-stream state, work planning and the
// host/device batch entry points.  Host code only; kernels live in jaad_lc.hip.
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdio>
#include <cstring>
#include <new>
#include <string>
#include <vector>

#include <algorithm>
#include <atomic>
#include <memory>
#include <chrono>
#include <condition_variable>
#include <cstdlib>
#include <functional>
#include <mutex>
#include <thread>

#include "jaad_lc.h"
#include "jaad_sbr.h"
#include "tables/jaad_sbr_tables.inc"
#include "tables/jaad_ps_tables.inc"
#include "tables/jaad_tables.inc"

using namespace jaad;

namespace {

// offset (in floats) into the SBR constant buffer of qmf32_pre_twiddle, after qmf_c | dct4 | noise
constexpr size_t kSbrConstTw32 = 640 + 224 + 1024;

// SampleFrequency maxTNS_SFB {long, short} (A/SampleFrequency.java:15-26)
const unsigned char kMaxTnsSfb[12][2] = {{31, 9}, {31, 9}, {34, 10}, {40, 14}, {42, 14}, {51, 14},
                                         {46, 14}, {46, 14}, {42, 14}, {42, 14}, {42, 14}, {39, 14}};

struct DevBuf {
    void* p = nullptr;
    size_t cap = 0;
    hipError_t ensure(size_t n)
    {
        if (n <= cap) return hipSuccess;
        if (p) (void)hipFree(p);
        p = nullptr;
        cap = 0;
        hipError_t e = hipMalloc(&p, n);
        if (e == hipSuccess) cap = n;
        return e;
    }
    void release()
    {
        if (p) (void)hipFree(p);
        p = nullptr;
        cap = 0;
    }
};

// page-locked host staging (grows, never shrinks)
struct PinnedBuf {
    void* p = nullptr;
    size_t cap = 0;
    hipError_t ensure(size_t n)
    {
        if (n <= cap) return hipSuccess;
        if (p) (void)hipHostFree(p);
        p = nullptr;
        cap = 0;
        const size_t want = n + n / 2;
        hipError_t e = hipHostMalloc(&p, want, hipHostMallocDefault);
        if (e == hipSuccess) cap = want;
        return e;
    }
    void release()
    {
        if (p) (void)hipHostFree(p);
        p = nullptr;
        cap = 0;
    }
};

// Host worker threads of a context: 16 (one GPU's CPU share on the target nodes) or fewer CPUs;
// JAAD_HOST_THREADS overrides (1..64).
static int host_threads()
{
    if (const char* e = std::getenv("JAAD_HOST_THREADS")) {
        const int v = std::atoi(e);
        if (v >= 1 && v <= 64) return v;
    }
    const unsigned hw = std::thread::hardware_concurrency();
    return (int)std::min(16u, hw ? hw : 1u);
}

// Persistent host workers for the per-call record build (fn(t) for t < size(); the caller runs
// t = 0), so a call does not pay thread start-up.
class WorkerPool {
public:
    explicit WorkerPool(int n) : n_(n < 1 ? 1 : n)
    {
        for (int t = 1; t < n_; t++) th_.emplace_back([this, t] { loop(t); });
    }
    ~WorkerPool()
    {
        {
            std::lock_guard<std::mutex> g(mu_);
            stop_ = true;
        }
        cv_.notify_all();
        for (auto& x : th_) x.join();
    }
    int size() const { return n_; }
    void run(const std::function<void(int)>& fn)
    {
        {
            std::lock_guard<std::mutex> g(mu_);
            fn_ = &fn;
            pending_ = n_ - 1;
            gen_++;
        }
        cv_.notify_all();
        fn(0);
        std::unique_lock<std::mutex> lk(mu_);
        done_.wait(lk, [this] { return pending_ == 0; });
        fn_ = nullptr;
    }

private:
    void loop(int t)
    {
        uint64_t seen = 0;
        for (;;) {
            const std::function<void(int)>* fn;
            {
                std::unique_lock<std::mutex> lk(mu_);
                cv_.wait(lk, [&] { return stop_ || gen_ != seen; });
                if (stop_) return;
                seen = gen_;
                fn = fn_;
            }
            (*fn)(t);
            {
                std::lock_guard<std::mutex> g(mu_);
                if (--pending_ == 0) done_.notify_one();
            }
        }
    }
    int n_;
    std::vector<std::thread> th_;
    std::mutex mu_;
    std::condition_variable cv_, done_;
    const std::function<void(int)>* fn_ = nullptr;
    uint64_t gen_ = 0;
    int pending_ = 0;
    bool stop_ = false;
};

// jaad_decode_batch pipeline: a batch is cut into up to kMaxPieces run-aligned pieces whose
// H2D copy, kernels and D2H copy overlap on three streams; pageable caller memory goes through
// kStageSlots page-locked staging slots per direction.
#ifndef JAAD_MAX_PIECES
#define JAAD_MAX_PIECES 12
#endif
#ifndef JAAD_MIN_PIECE_FRAMES
#define JAAD_MIN_PIECE_FRAMES 2048
#endif
constexpr int kMaxPieces = JAAD_MAX_PIECES, kStageSlots = 2;
enum : int { kPinRegistered = 0, kPinForeign = 1, kPinOwned = 2 };
constexpr int kMaxElements = 8;

// Channel elements of the AAC-LC channel configurations 3..7 (ISO/IEC 14496-3 Table 1.19: C, L/R,
// surrounds, LFE), channels per element; returns the element count (0: not a multichannel config)
int mc_elements(int channel_config, uint8_t* nch)
{
    static const uint8_t kLayouts[5][6] = {{1, 2}, {1, 2, 1}, {1, 2, 2}, {1, 2, 2, 1}, {1, 2, 2, 2, 1}};
    static const int kCount[5] = {2, 3, 3, 4, 5};
    if (channel_config < 3 || channel_config > 7) return 0;
    const int k = channel_config - 3;
    for (int i = 0; i < kCount[k]; i++) nch[i] = kLayouts[k][i];
    return kCount[k];
}
// the LFE position of a multichannel layout: configurations 6 and 7 end with the LFE
bool mc_is_lfe(int channel_config, int k, int n) { return (channel_config == 6 || channel_config == 7) && k == n - 1; }
constexpr uint32_t kMinPieceFrames = JAAD_MIN_PIECE_FRAMES;

// One call's SBR/PS parameter records: built on the host straight into page-locked staging,
// copied on the context's copy stream while the previous call's kernels run.  Two sets
// alternate between calls; `copied` guards the staging, `used` the device copy.
//   part 1: recs | psf | chunks | last | runs
//   part 2: one E_orig region per worker (sized for the worst case, only the used prefix is
//           uploaded) | tabs
struct RecSet {
    PinnedBuf h1, h2;
    DevBuf d1, d2;
    hipEvent_t copied = nullptr, used = nullptr;
    bool live = false;
};

}  // namespace

struct jaad_ctx {
    jaad_stream_cfg cfg{};
    int device = 0;
    int nch = 2;                 // channel-frame records per frame (a multichannel config: all channels)
    // channel elements of a frame, in bitstream order (SyntacticElements.process,
    // A/syntax/SyntacticElements.java:235-248): 1 = SCE/LFE, 2 = CPE; one element for channel
    // configurations 1 and 2
    int n_elem = 1, n_cpe = 0;
    uint8_t elem_nch[kMaxElements] = {};
    uint32_t n_slots = 0;
    hipStream_t stream = nullptr;
    float* d_state[2] = {nullptr, nullptr};  // [slot][2][1024], double-buffered (see plan())
    int parity = 0;                          // d_state[parity] holds the current state
    LdsTables* d_tables = nullptr;
    GlobalTables* d_gtab = nullptr;
    float* d_iq = nullptr;
    DevBuf d_batch, d_pcm;
    // the chunk table (+ skip list) of the current plan: two slots, so that a new plan (the launch
    // pipeline re-plans every piece) does not wait for the kernels of the previous one
    DevBuf d_chunks[2];
    PinnedBuf h_chunks[2];                   // staging of each slot's upload
    hipEvent_t chunks_copied[2] = {};        // h_chunks[i] may be rewritten once this has completed
    bool chunks_live[2] = {false, false};
    hipEvent_t chunks_read[2] = {};          // d_chunks[i] may be rewritten once this has completed (recorded
    bool chunks_read_live[2] = {false, false};  // when plan() left slot i; round 6)
    int chunk_slot = 0;                      // slot of the current plan
    bool hint_short = false;                 // the current call's batch holds EIGHT_SHORT frames (KernelArgs::short_pair)
    // Every call's device work (whatever stream it is queued on) waits for the previous call's
    // `done`: the chunk table, the double-buffered state and the SBR/PS state are reused call
    // after call.  The state_* entry points and jaad_wait wait for it too.
    hipEvent_t done = nullptr;
    bool done_live = false;
    hipStream_t last_stream = nullptr;  // stream of the previous device call
    std::vector<ChunkDesc> chunks;
    std::vector<uint32_t> plan_slots, plan_begin;  // plan cache key
    // dropped frames (jaad_batch.frame_status): the call's kept batch frames in order (virtual
    // frame -> batch frame), the runs' first virtual frames, and the runs of dropped frames as
    // (first, count) pairs + sentinel (KernelArgs::skips: uploaded behind the chunk table, and
    // part of the plan cache key).  d_skips: a copy for the multichannel HE-AAC interleave.
    std::vector<uint32_t> keep, vbegin, skips, plan_skips;
    DevBuf d_skips;
    PinnedBuf h_skips;
    hipEvent_t skips_copied = nullptr;
    bool skips_live = false;
    uint32_t plan_n_chunks = 0;  // skip list offset in d_chunks (ChunkDesc units)
    std::vector<uint8_t> slot_used;
    bool plan_valid = false;
    int n_cu = 256;
    uint32_t lc_waves = 0;       // LC kernel waves resident on the whole device (one per chunk)
    uint32_t chunk_frames = 0;   // 0 = size chunks from lc_waves; JAAD_CHUNK_FRAMES overrides
    uint32_t syn_frames = 0;     // 0 = kSbrSynFrames frames per synthesis chunk; JAAD_SYN_FRAMES overrides
    float* dbg = nullptr;
    int dbg_frame = 0;
    std::string err;
    // ---- SBR (cfg.sbr) ----
    std::unique_ptr<SbrHost> sbr_host;
    std::vector<SbrHostSlot> sbr_slots;          // parameter-side state per slot (host)
    std::vector<uint32_t> sbr_depth;             // HF fix pass of each channel-frame (scratch)
    SbrChState* d_sbr_state = nullptr;           // [slot][2], rewritten at the end of each call
    float* d_sbr_const = nullptr;                // qmf_c[640] | dct4 tab[192] w_re[16] w_im[16] | noise[1024] |
                                                 // qmf32_pre_twiddle[32][2]
    DevBuf d_time, d_xlow, d_xsyn, d_xcarry, d_gq;
    hipStream_t cstream = nullptr;               // record uploads
    hipStream_t rec_stream = nullptr;            // (the launch pipeline: uploads on its H2D stream)
    RecSet rsets[2];
    int rset = 0;
    std::unique_ptr<WorkerPool> workers;
    std::vector<SbrChunk> sbr_chunks;
    std::vector<uint32_t> sbr_last;
    std::vector<uint32_t> sbr_rbegin, sbr_fmap, sbr_ups;  // record plan of the call (launch_sbr_stage)
    float* sbr_dbg = nullptr;
    // ---- PS (cfg.ps) ----
    PsState* d_ps_state = nullptr;               // [slot]
    PsConst* d_ps_const = nullptr;
    float* d_ps_zero = nullptr;  // SbrArgs::zero (behind d_ps_const, one allocation)
    DevBuf d_xps, d_xhl, d_xhr, d_pg, d_hb;
    std::vector<uint32_t> ps_runs;
    // ---- host-buffer entry (jaad_decode_batch), set up on its first call ----
    hipStream_t h2d = nullptr, d2h = nullptr;      // copy streams beside `stream` (one DMA engine each)
    hipEvent_t ev_in[kMaxPieces] = {}, ev_k[kMaxPieces] = {}, ev_out[kMaxPieces] = {};
    PinnedBuf stage_in[kStageSlots], stage_out[kStageSlots];
    // the launch pipeline's roll-back copies (device: core overlap, SBR and PS state of every slot)
    DevBuf d_backup;
    uint32_t sbr_pieces = 0;  // JAAD_SBR_PIECES (tuning): pieces of a launch-pipeline call
    DevBuf d_flag;                                 // |q| check result of a host-buffer call (device)
    PinnedBuf h_flag;
    DevBuf d_cce;                                  // coupling: term offsets / meta / gains, then addends
    PinnedBuf h_cce;                               // their host image
    std::unique_ptr<WorkerPool> io;                // validation / staging copies
    struct PinRange {
        uintptr_t p;
        size_t n;
        int kind;  // kPinRegistered (hipHostRegister'd here), kPinForeign (already page-locked), kPinOwned (jaad_host_alloc)
    };
    std::vector<PinRange> pinned;  // jaad_host_register / jaad_host_alloc ranges
    uint32_t plan_L = 0;                           // chunk length of the cached plan
    // ---- multichannel HE-AAC (configurations 3..7 with cfg.sbr): every channel element runs as its
    // own mono (SCE, LFE) or stereo (CPE) SBR context on the element's records, gathered from the
    // batch; the elements' PCM is then interleaved (launch_mc_sbr) ----
    std::vector<jaad_ctx*> children;
    DevBuf d_mc;                                   // gathered element records + element PCM
    std::vector<jaad_sbr_frame> h_mc_sbr;          // one element's SBR records of the call
    std::vector<jaad_cce_term> h_mc_terms;         // one element's coupling terms of the call
};

namespace jaad {

void build_lds_tables(int sf_index, LdsTables* t, GlobalTables* gt)
{
    std::memset(t, 0, sizeof(*t));
    std::memset(gt, 0, sizeof(*gt));
    const float* LW[2] = {JAAD_SINE_1024, JAAD_KBD_1024};
    for (int sh = 0; sh < 2; sh++)
        for (int o = 0; o < 16; o++)
            for (int u = 0; u < 64; u++) t->win_pair[sh][o >> 1][u][o & 1] = LW[sh][long_pos_host(u, o)];
    std::memcpy(t->win_short[0], JAAD_SINE_128, sizeof(t->win_short[0]));
    std::memcpy(t->win_short[1], JAAD_KBD_128, sizeof(t->win_short[1]));
    std::memcpy(t->mdct_l, JAAD_MDCT_TABLE_2048, sizeof(t->mdct_l));
    for (int s = 0; s < 8; s++)
        for (int u = 0; u < 64; u++) {
            t->mdct_post[s][u][0] = JAAD_MDCT_TABLE_2048[lane_pos_host(u) + 64 * s][0];
            t->mdct_post[s][u][1] = JAAD_MDCT_TABLE_2048[lane_pos_host(u) + 64 * s][1];
            t->mdct_post_f[s][u][0] = t->mdct_post[s][u][0] * (1.0f / 32767.0f);
            t->mdct_post_f[s][u][1] = t->mdct_post[s][u][1] * (1.0f / 32767.0f);
        }
    for (int sh = 0; sh < 2; sh++)
        for (int o = 0; o < 16; o++)
            for (int u = 0; u < 64; u++) {
                const int P = long_pos_host(u, o);
                t->win_ss[sh][o >> 1][u][o & 1] = P < 448 ? 0.0f : P < 576 ? (sh ? JAAD_KBD_128 : JAAD_SINE_128)[P - 448] : 1.0f;
            }
    for (int k = 0; k < 64; k++) {
        t->mdct_s_f[k][0] = JAAD_MDCT_TABLE_128[k][0] * (1.0f / 32767.0f);
        t->mdct_s_f[k][1] = JAAD_MDCT_TABLE_128[k][1] * (1.0f / 32767.0f);
    }
    // 512-point IFFT twiddles roots[k*m] (FFT.java:116-120, inverse column 1) pre-arranged per
    // register pass: pass 1 (i = 4, m = 64); pass 2 by b = position mod 8: slot 0 -> stage 8
    // (m = 32, k = b), slots 1,2 -> stage 16 (m = 16, k = b + 8e), slots 3..6 -> stage 32 (m = 8,
    // k = b + 8s); pass 3 by lane u, position p = lane_pos(u): slot 0 -> stage 64 (m = 4, k = p),
    // 1,2 -> stage 128 (m = 2, k = p + 64e), 3..6 -> stage 256 (m = 1, k = p + 64s)
    auto root = [](int idx, float* d) {
        d[0] = JAAD_FFT_TABLE_512[idx][0];
        d[1] = JAAD_FFT_TABLE_512[idx][1];
    };
    for (int k = 0; k < 4; k++) root(k * 64, t->tw1[k]);
    for (int b = 0; b < 8; b++) {
        root(32 * b, t->tw2[0][b]);
        for (int e = 0; e < 2; e++) root(16 * (b + 8 * e), t->tw2[1 + e][b]);
        for (int s = 0; s < 4; s++) root(8 * (b + 8 * s), t->tw2[3 + s][b]);
    }
    for (int u = 0; u < 64; u++) {  // pass 3: j = 0 -> 4p, j = 1,2 -> 2(p + 64e), j = 3..6 -> p + 64s
        const int p = lane_pos_host(u);
        root(4 * p, t->tw3[0][u]);
        for (int e = 0; e < 2; e++) root(2 * (p + 64 * e), t->tw3[1 + e][u]);
        for (int s = 0; s < 4; s++) root(p + 64 * s, t->tw3[3 + s][u]);
    }
    // radix-8 twiddles of the +-1 LSB kernel (jaad_lc.hip fft_r8_pass): register r holds the
    // sub-transform bitrev3(r) of its pass
    for (int r = 1; r < 8; r++) {
        const int m = ((r & 1) << 2) | (r & 2) | ((r >> 2) & 1);
        for (int b = 0; b < 8; b++) root(8 * m * b, t->tw2f[r - 1][b]);
        for (int u = 0; u < 64; u++) root(m * lane_pos_host(u), t->tw3f[r - 1][u]);
    }
    std::memcpy(t->mdct_s, JAAD_MDCT_TABLE_128, sizeof(t->mdct_s));
    for (int k = 0; k < 32; k++) {
        t->roots_s[k][0] = JAAD_FFT_TABLE_64[k][0];
        t->roots_s[k][1] = JAAD_FFT_TABLE_64[k][1];
    }
    for (int i = 0; i < 256; i++) t->sf_gain[i] = JAAD_SCALEFACTOR_TABLE[100 + i];
    for (int i = 0; i < 2 * kIqHead; i++) {
        const int q = i - kIqHead;  // float of (q>0 ? IQ[q] : -IQ[-q]): q = 0 gives -0.0
        t->iq_signed[i] = q > 0 ? JAAD_IQ_TABLE[q] : -JAAD_IQ_TABLE[-q];
    }
    std::memcpy(gt->tns_coef[0], JAAD_TNS_COEF_0_3, sizeof(JAAD_TNS_COEF_0_3));
    std::memcpy(gt->tns_coef[1], JAAD_TNS_COEF_0_4, sizeof(JAAD_TNS_COEF_0_4));
    std::memcpy(gt->tns_coef[2], JAAD_TNS_COEF_1_3, sizeof(JAAD_TNS_COEF_1_3));
    std::memcpy(gt->tns_coef[3], JAAD_TNS_COEF_1_4, sizeof(JAAD_TNS_COEF_1_4));
    const short* L = JAAD_SWB_OFFSET_LONG_WINDOW[sf_index];
    const short* S = JAAD_SWB_OFFSET_SHORT_WINDOW[sf_index];
    t->nswb_l = JAAD_SWB_LONG_WINDOW_COUNT[sf_index];
    t->nswb_s = JAAD_SWB_SHORT_WINDOW_COUNT[sf_index];
    for (int i = 0; i <= t->nswb_l; i++) gt->swb_l[i] = L[i];
    for (int i = 0; i <= t->nswb_s; i++) gt->swb_s[i] = S[i];
    std::memset(t->quad2band_l, 255, sizeof(t->quad2band_l));
    std::memset(t->quad2band_s, 255, sizeof(t->quad2band_s));
    for (int b = 0; b < t->nswb_l; b++)
        for (int p = L[b]; p < L[b + 1]; p += 4) t->quad2band_l[p >> 2] = (uint8_t)b;
    for (int b = 0; b < t->nswb_s; b++)
        for (int p = S[b]; p < S[b + 1]; p += 4) t->quad2band_s[p >> 2] = (uint8_t)b;
    t->tns_max_l = kMaxTnsSfb[sf_index][0];
    t->tns_max_s = kMaxTnsSfb[sf_index][1];
}

}  // namespace jaad

namespace {

int fail(jaad_ctx* c, hipError_t e, const char* what)
{
    if (c) {
        c->err = std::string(what) + ": " + hipGetErrorString(e);
    }
    return JAAD_ERR_HIP;
}

#define HIPCHK(call)                                 \
    do {                                             \
        hipError_t e_ = (call);                      \
        if (e_ != hipSuccess) return fail(ctx, e_, #call); \
    } while (0)

// JAAD_SYNC_LAUNCHES=1 (diagnostics only): each launch group is followed by a synchronize of its
// stream, so that a device fault is reported against the launch that raised it rather than at a
// later copy (the error text names the launch call)
bool sync_launches()
{
    static const bool on = [] {
        const char* e = std::getenv("JAAD_SYNC_LAUNCHES");
        return e && e[0] == '1';
    }();
    return on;
}
#define LAUNCHCHK(call, strm)                                                   \
    do {                                                                        \
        HIPCHK(call);                                                           \
        if (sync_launches()) {                                                  \
            hipError_t s_ = hipStreamSynchronize(strm);                         \
            if (s_ != hipSuccess) return fail(ctx, s_, "after " #call);         \
        }                                                                       \
    } while (0)

int validate_cfg(const jaad_stream_cfg* cfg)
{
    if (!cfg) return JAAD_ERR_INVALID_ARG;
    if (cfg->abi_version != JAAD_ABI_VERSION) return JAAD_ERR_ABI;
    if (cfg->profile != 2) return JAAD_ERR_UNSUPPORTED;  // Profile.AAC_LC (A/Profile.java)
    if (cfg->sf_index > 11) return JAAD_ERR_UNSUPPORTED;
    if (cfg->channel_config < 1 || cfg->channel_config > 7) return JAAD_ERR_UNSUPPORTED;
    // multichannel: AAC-LC elements, or SBR per element (HE-AAC v1); PS only in a mono stream
    if (cfg->channel_config > 2 && cfg->ps) return JAAD_ERR_UNSUPPORTED;
    if (cfg->tns_mode > JAAD_TNS_SPEC) return JAAD_ERR_INVALID_ARG;
    if (cfg->precision > JAAD_PRECISION_LSB1) return JAAD_ERR_INVALID_ARG;
    if (cfg->sbr > 1 || cfg->ps > 1) return JAAD_ERR_UNSUPPORTED;
    if (cfg->ps && (!cfg->sbr || cfg->channel_config != 1)) return JAAD_ERR_UNSUPPORTED;
    // SBR at twice the core rate (bs_samplerate_mode = 1, A/sbr/SBR.java:105), or downsampled
    // (extension rate = core rate: SBR.downSampled, 32-band synthesis, A/sbr/SBR.java:35-37,100)
    if (cfg->sbr && cfg->ext_sf_index != cfg->sf_index && (cfg->sf_index < 3 || cfg->ext_sf_index + 3 != cfg->sf_index))
        return JAAD_ERR_UNSUPPORTED;
    return JAAD_OK;
}

// (Re)build the chunk table for the batch's runs; cached when the run layout repeats.  The new
// table is built in locals and committed (cache key, slot_used, device copy) only once it is
// complete, so a rejected batch leaves the previous plan intact.  The upload is queued on the
// call's stream (ordered after the previous call by launch()) from page-locked staging.
// `size_frames` (0: the batch's) is the frame count one launch covers: the host-buffer entry
// launches the kernel once per piece of the batch, so its chunks are sized for a piece.
// device chunk table of the current plan
const ChunkDesc* chunks_dev(const jaad_ctx* ctx) { return static_cast<const ChunkDesc*>(ctx->d_chunks[ctx->chunk_slot].p); }

// b: the planner's view of the call (with dropped frames: keep_map's virtual batch, the kept
// frames numbered consecutively); the chunks it writes hold batch frames (ctx->keep translates
// them when ctx->skips is not empty, the skip list then follows the chunk table on the device)
int plan(jaad_ctx* ctx, const jaad_batch* b, hipStream_t stream, uint32_t size_frames = 0)
{
    if (!b->stream_slot || !b->frame_begin) return JAAD_ERR_INVALID_ARG;
    if (b->frame_begin[0] != 0 || b->frame_begin[b->n_runs] != b->n_frames) return JAAD_ERR_INVALID_ARG;
    // One wave decodes one chunk; a chunk that does not start its run re-decodes one frame.
    // Chunk length L is chosen so that the chunks fill the device's resident waves about once
    // (balanced, no tail round), but never shorter than kMinChunkFrames (prefix overhead).
    uint32_t L = ctx->chunk_frames;
    if (!L) {
        const uint64_t cap = ctx->lc_waves ? ctx->lc_waves : 4096;
        const uint64_t n = size_frames ? size_frames : b->n_frames;
        L = (uint32_t)std::max<uint64_t>(kMinChunkFrames, (n + cap - 1) / cap);
    }
    L = std::min<uint32_t>(L, 0xffff);
    bool same = ctx->plan_valid && ctx->plan_L == L && ctx->plan_slots.size() == b->n_runs &&
                std::memcmp(ctx->plan_slots.data(), b->stream_slot, b->n_runs * sizeof(uint32_t)) == 0 &&
                std::memcmp(ctx->plan_begin.data(), b->frame_begin, (b->n_runs + 1) * sizeof(uint32_t)) == 0 &&
                ctx->plan_skips == ctx->skips;
    if (same) return JAAD_OK;
    std::vector<ChunkDesc> chunks;
    std::vector<uint8_t> used(ctx->n_slots, 0);
    for (uint32_t r = 0; r < b->n_runs; r++) {
        uint32_t f0 = b->frame_begin[r], f1 = b->frame_begin[r + 1];
        uint32_t slot = b->stream_slot[r];
        if (f1 < f0 || slot >= ctx->n_slots) return JAAD_ERR_INVALID_ARG;
        if (used[slot]) return JAAD_ERR_INVALID_ARG;  // one run per stream per call
        used[slot] = 1;
        if (f1 == f0) {  // empty run: carry the state over unchanged
            chunks.push_back(ChunkDesc{f0, kChunkLoadState | kChunkStoreState, slot, 0});
            continue;
        }
        // split the run into `parts` chunks of equal length (+-1 frame)
        const uint32_t len = f1 - f0, parts = (len + L - 1) / L;
        for (uint32_t i = 0; i < parts; i++) {
            const uint32_t f = f0 + (uint32_t)((uint64_t)len * i / parts);
            const uint32_t fe = f0 + (uint32_t)((uint64_t)len * (i + 1) / parts);
            uint32_t info = fe - f;
            info |= (f == f0) ? kChunkLoadState : kChunkPrefix;
            if (fe == f1) info |= kChunkStoreState;
            chunks.push_back(ChunkDesc{f, info, slot, 0});
        }
    }
    // Self-check of the table before it can reach a launch (round 6): every chunk's
    // slot in range, its frames (the re-decoded prefix frame included) inside its run's frames of the
    // planner's view, and with dropped frames its walk inside the kept-frame map and its first skip
    // entry inside the list.  O(chunks); a failure is an internal error, never a launch.
    {
        const uint32_t nv = b->n_frames;
        for (const ChunkDesc& c : chunks) {
            const uint32_t n = c.info & 0xffff, pre = (c.info & kChunkPrefix) ? 1u : 0u;
            const bool ok = c.slot < ctx->n_slots && (n == 0 || (c.frame0 >= pre && (uint64_t)c.frame0 + n <= nv)) &&
                            (ctx->skips.empty() || n == 0 || (uint64_t)c.frame0 + n <= ctx->keep.size());
            if (!ok) {
                ctx->err = "internal: chunk table out of range (frame " + std::to_string(c.frame0) + ", " +
                           std::to_string(n) + " frames, slot " + std::to_string(c.slot) + ")";
                return JAAD_ERR_INVALID_ARG;
            }
        }
    }
    if (!ctx->skips.empty()) {  // virtual frames -> batch frames; each chunk's first skip entry
        const std::vector<uint32_t>& k = ctx->keep;
        const uint32_t ns = (uint32_t)ctx->skips.size() / 2;  // incl. the sentinel
        for (ChunkDesc& c : chunks) {
            if ((c.info & 0xffff) == 0) continue;  // empty run: no frame is read
            const uint32_t v0 = c.frame0 - ((c.info & kChunkPrefix) ? 1 : 0);
            c.frame0 = k[v0];
            uint32_t lo = 0, hi = ns - 1;  // first run of dropped frames starting after frame0
            while (lo < hi) {
                const uint32_t m = (lo + hi) / 2;
                if (ctx->skips[2 * m] <= c.frame0) lo = m + 1;
                else hi = m;
            }
            c.skip = lo;
        }
    } else {
        for (ChunkDesc& c : chunks) c.frame0 -= (c.info & kChunkPrefix) ? 1 : 0;
    }
    ctx->plan_valid = false;  // from here on the cached layout no longer describes d_chunks
    const size_t cbytes = chunks.size() * sizeof(ChunkDesc);
    const size_t bytes = cbytes + ctx->skips.size() * sizeof(uint32_t);
    const int slot = ctx->chunk_slot ^ 1;  // (the current plan's slot may still be read by queued kernels)
    if (ctx->chunks_live[slot]) HIPCHK(hipEventSynchronize(ctx->chunks_copied[slot]));  // staging in use?
    // Every LC launch that read the current plan's table was queued by an earlier call or piece
    // (this one is ordered after them on `stream`, launch()), so an event here marks the end of
    // its readers; the other slot's readers ended at the event recorded when it was left, which
    // its upload waits for on the device (a reallocation of the table on the host: hipFree under
    // a running kernel).  One event per plan switch, none per call.
    HIPCHK(hipEventRecord(ctx->chunks_read[ctx->chunk_slot], stream));
    ctx->chunks_read_live[ctx->chunk_slot] = true;
    if (ctx->chunks_read_live[slot]) {
        if (bytes + 16 > ctx->d_chunks[slot].cap) HIPCHK(hipEventSynchronize(ctx->chunks_read[slot]));
        else HIPCHK(hipStreamWaitEvent(stream, ctx->chunks_read[slot], 0));
    }
    HIPCHK(ctx->h_chunks[slot].ensure(bytes + 16));
    HIPCHK(ctx->d_chunks[slot].ensure(bytes + 16));
    if (bytes) {
        std::memcpy(ctx->h_chunks[slot].p, chunks.data(), cbytes);
        if (!ctx->skips.empty())
            std::memcpy(static_cast<char*>(ctx->h_chunks[slot].p) + cbytes, ctx->skips.data(), bytes - cbytes);
        HIPCHK(hipMemcpyAsync(ctx->d_chunks[slot].p, ctx->h_chunks[slot].p, bytes, hipMemcpyHostToDevice, stream));
        HIPCHK(hipEventRecord(ctx->chunks_copied[slot], stream));
        ctx->chunks_live[slot] = true;
    }
    ctx->chunk_slot = slot;
    ctx->chunks.swap(chunks);
    ctx->slot_used.swap(used);
    ctx->plan_slots.assign(b->stream_slot, b->stream_slot + b->n_runs);
    ctx->plan_begin.assign(b->frame_begin, b->frame_begin + b->n_runs + 1);
    ctx->plan_L = L;
    ctx->plan_skips = ctx->skips;
    ctx->plan_n_chunks = (uint32_t)ctx->chunks.size();
    ctx->plan_valid = true;
    return JAAD_OK;
}

// wait (host) until every call queued on the context so far has finished on the device
int sync_ctx(jaad_ctx* ctx)
{
    HIPCHK(hipSetDevice(ctx->device));
    if (ctx->done_live) HIPCHK(hipEventSynchronize(ctx->done));
    HIPCHK(hipStreamSynchronize(ctx->stream));
    return JAAD_OK;
}

// Dropped frames (jaad_batch.frame_status, A/Decoder.java:89-101): the kernels of the call walk
// the kept frames only.  `vb` becomes the planner's view of the batch (the kept frames numbered
// consecutively, runs in the same order and slots); ctx->keep maps them back to batch frames and
// ctx->skips lists the runs of dropped frames (empty when nothing is dropped), which plan() turns
// into batch-frame chunks and the device skip list.
int keep_map(jaad_ctx* ctx, const jaad_batch* b, jaad_batch& vb)
{
    vb = *b;
    ctx->skips.clear();
    if (!b->frame_status) return JAAD_OK;
    if (!b->stream_slot || !b->frame_begin) return JAAD_ERR_INVALID_ARG;
    if (b->frame_begin[0] != 0 || b->frame_begin[b->n_runs] != b->n_frames) return JAAD_ERR_INVALID_ARG;
    std::vector<uint32_t>& keep = ctx->keep;
    std::vector<uint32_t>& vbeg = ctx->vbegin;
    keep.clear();
    vbeg.assign(1, 0);
    for (uint32_t r = 0; r < b->n_runs; r++) {
        if (b->frame_begin[r + 1] < b->frame_begin[r]) return JAAD_ERR_INVALID_ARG;
        for (uint32_t f = b->frame_begin[r]; f < b->frame_begin[r + 1]; f++)
            if (b->frame_status[f] == JAAD_FRAME_DECODE) keep.push_back(f);
        vbeg.push_back((uint32_t)keep.size());
    }
    vb.n_frames = (uint32_t)keep.size();
    vb.frame_begin = vbeg.data();
    if (keep.size() == b->n_frames) return JAAD_OK;  // nothing dropped
    for (uint32_t f = 0; f < b->n_frames;) {
        if (b->frame_status[f] == JAAD_FRAME_DECODE) {
            f++;
            continue;
        }
        uint32_t e = f + 1;
        while (e < b->n_frames && b->frame_status[e] != JAAD_FRAME_DECODE) e++;
        ctx->skips.push_back(f);
        ctx->skips.push_back(e - f);
        f = e;
    }
    ctx->skips.push_back(UINT32_MAX);  // sentinel: never the frame after a kept one
    ctx->skips.push_back(0);
    return JAAD_OK;
}

// device copy of ctx->skips for a launch that plans no LC chunks itself (the multichannel HE-AAC
// interleave); null when nothing is dropped
int upload_skips(jaad_ctx* ctx, hipStream_t stream, const uint32_t** d)
{
    *d = nullptr;
    if (ctx->skips.empty()) return JAAD_OK;
    const size_t bytes = ctx->skips.size() * sizeof(uint32_t);
    if (ctx->skips_live) HIPCHK(hipEventSynchronize(ctx->skips_copied));  // staging in use?
    HIPCHK(ctx->h_skips.ensure(bytes));
    HIPCHK(ctx->d_skips.ensure(bytes));
    std::memcpy(ctx->h_skips.p, ctx->skips.data(), bytes);
    HIPCHK(hipMemcpyAsync(ctx->d_skips.p, ctx->h_skips.p, bytes, hipMemcpyHostToDevice, stream));
    HIPCHK(hipEventRecord(ctx->skips_copied, stream));
    ctx->skips_live = true;
    *d = static_cast<const uint32_t*>(ctx->d_skips.p);
    return JAAD_OK;
}

// the device skip list behind the chunk table of the current plan (null: nothing dropped)
const uint32_t* plan_skips_dev(const jaad_ctx* ctx)
{
    if (ctx->plan_skips.empty()) return nullptr;
    return reinterpret_cast<const uint32_t*>(chunks_dev(ctx) + ctx->plan_n_chunks);
}

uint32_t n_skip_runs(const jaad_ctx* ctx) { return ctx->skips.empty() ? 0u : (uint32_t)ctx->skips.size() / 2 - 1; }

bool frame_dropped(const jaad_batch* b, size_t f) { return b->frame_status && b->frame_status[f] != JAAD_FRAME_DECODE; }

bool sbr_downsampled(const jaad_stream_cfg& c) { return c.sbr && c.ext_sf_index == c.sf_index; }

size_t pcm_bytes_per_frame(const jaad_ctx* ctx, uint32_t flags)
{
    return jaad_frame_pcm_bytes(&ctx->cfg, flags);
}

// slots a call does not touch keep their state: carry them into the other parity buffer
template <typename T>
int carry_untouched(jaad_ctx* ctx, T* out, const T* in, size_t per_slot, hipStream_t stream)
{
    for (uint32_t s = 0; s < ctx->n_slots;) {
        if (ctx->slot_used[s]) {
            s++;
            continue;
        }
        uint32_t e = s;
        while (e < ctx->n_slots && !ctx->slot_used[e]) e++;
        HIPCHK(hipMemcpyAsync(out + (size_t)s * per_slot, in + (size_t)s * per_slot, (e - s) * per_slot * sizeof(T),
                              hipMemcpyDeviceToDevice, stream));
        s = e;
    }
    return JAAD_OK;
}

static_assert(sizeof(jaad_ps_frame) == 528 && sizeof(jaad_sbr_frame) == 1968, "jaad_gpu.h record sizes");

// PS parameters the Java parser can produce (A/ps/PSImpl.java:103-199): borders 0 = b_0 < .. <
// b_num_env = 32, |IID| <= num_steps, ICC and IPD/OPD in 0..7, nr_ipdopd_par 0 / 11 / 17.  A frame
// without PS data is decoded as SBR1.process does then: mono, copied to the right channel
// (A/sbr/SBR1.java:75-81); the PS state waits for the next PS frame.
static bool ps_frame_ok(const jaad_sbr_frame& F)
{
    const jaad_ps_frame& p = F.ps;
    if (!F.ps_present) return true;
    if (p.num_env < 1 || p.num_env > 5 || p.iid_mode > 5 || p.icc_mode > 5) return false;
    if (p.nr_ipdopd_par != 0 && p.nr_ipdopd_par != 11 && p.nr_ipdopd_par != 17) return false;
    if (p.border[0] != 0 || p.border[p.num_env] != 32) return false;
    for (int e = 0; e < p.num_env; e++)
        if (p.border[e + 1] <= p.border[e]) return false;
    const int steps = p.iid_mode >= 3 ? 15 : 7;
    for (int e = 0; e < p.num_env; e++)
        for (int b = 0; b < 20; b++)
            if (p.iid[e][b] > steps || p.iid[e][b] < -steps || p.icc[e][b] < 0 || p.icc[e][b] > 7) return false;
    for (int e = 0; e < p.num_env; e++)
        for (int b = 0; b < p.nr_ipdopd_par; b++)
            if (p.ipd[e][b] < 0 || p.ipd[e][b] > 7 || p.opd[e][b] < 0 || p.opd[e][b] > 7) return false;
    return true;
}

static void build_ps_const(PsConst* k)
{
    std::memset(k, 0, sizeof *k);
    std::memcpy(k->phi_qmf, JAAD_PS_PHI_FRACT_QMF, sizeof k->phi_qmf);
    std::memcpy(k->phi_sub, JAAD_PS_PHI_FRACT_SUBQMF20, sizeof k->phi_sub);
    std::memcpy(k->q_qmf, JAAD_PS_Q_FRACT_ALLPASS_QMF, sizeof k->q_qmf);
    std::memcpy(k->q_sub, JAAD_PS_Q_FRACT_ALLPASS_SUBQMF20, sizeof k->q_sub);
    std::memcpy(k->filter_a, JAAD_PS_FILTER_A, sizeof k->filter_a);
    std::memcpy(k->sf_iid[0], JAAD_PS_SF_IID_NORMAL, sizeof JAAD_PS_SF_IID_NORMAL);
    std::memcpy(k->sf_iid[1], JAAD_PS_SF_IID_FINE, sizeof JAAD_PS_SF_IID_FINE);
    std::memcpy(k->cos_alphas, JAAD_PS_COS_ALPHAS, sizeof k->cos_alphas);
    std::memcpy(k->sin_alphas, JAAD_PS_SIN_ALPHAS, sizeof k->sin_alphas);
    std::memcpy(k->cos_betas[0], JAAD_PS_COS_BETAS_NORMAL, sizeof JAAD_PS_COS_BETAS_NORMAL);
    std::memcpy(k->cos_betas[1], JAAD_PS_COS_BETAS_FINE, sizeof JAAD_PS_COS_BETAS_FINE);
    std::memcpy(k->sin_betas[0], JAAD_PS_SIN_BETAS_NORMAL, sizeof JAAD_PS_SIN_BETAS_NORMAL);
    std::memcpy(k->sin_betas[1], JAAD_PS_SIN_BETAS_FINE, sizeof JAAD_PS_SIN_BETAS_FINE);
    // IIDMode hands (sin_gammas, cos_gammas) to IIDTables(cos_gammas, sin_gammas): swapped
    // (A/ps/IIDMode.java:16-28, A/ps/IIDTables.java:17-21)
    std::memcpy(k->cos_gammas[0], JAAD_PS_SIN_GAMMAS_NORMAL, sizeof JAAD_PS_SIN_GAMMAS_NORMAL);
    std::memcpy(k->cos_gammas[1], JAAD_PS_SIN_GAMMAS_FINE, sizeof JAAD_PS_SIN_GAMMAS_FINE);
    std::memcpy(k->sin_gammas[0], JAAD_PS_COS_GAMMAS_NORMAL, sizeof JAAD_PS_COS_GAMMAS_NORMAL);
    std::memcpy(k->sin_gammas[1], JAAD_PS_COS_GAMMAS_FINE, sizeof JAAD_PS_COS_GAMMAS_FINE);
    std::memcpy(k->sincos_b[0], JAAD_PS_SINCOS_ALPHAS_B_NORMAL, sizeof JAAD_PS_SINCOS_ALPHAS_B_NORMAL);
    std::memcpy(k->sincos_b[1], JAAD_PS_SINCOS_ALPHAS_B_FINE, sizeof JAAD_PS_SINCOS_ALPHAS_B_FINE);
    std::memcpy(k->p8, JAAD_PS_P8_13_20, sizeof k->p8);
    std::memcpy(k->p2, JAAD_PS_P2_13_20, sizeof k->p2);
    std::memcpy(k->ipdopd_cos, JAAD_PS_IPDOPD_COS, sizeof k->ipdopd_cos);
    std::memcpy(k->ipdopd_sin, JAAD_PS_IPDOPD_SIN, sizeof k->ipdopd_sin);
}

// SBR: host records in stream order, chunk plan, then the SBR kernel over the core time samples
int launch_sbr_stage(jaad_ctx* ctx, const jaad_batch* b, void* pcm, uint32_t flags, hipStream_t stream)
{
    const int nch = ctx->nch;
    const bool ps = ctx->cfg.ps != 0;
    const int och = ps ? 2 : nch;  // channels of the QMF synthesis
    const size_t nf = b->n_frames;
    auto al = [](size_t x) { return (x + 255) & ~(size_t)255; };

    // The SBR stages run on the frames whose SBR data is usable, compacted per run ("records"):
    // a JAAD_SBR_UPSAMPLE frame skips SBR in the reference (A/syntax/CPE.java:196-204,
    // SCE.java:123-132), so the record before and after it are consecutive as far as the SBR
    // state goes.  Its PCM is the upsampled core (sbr_upsample_kernel).
    std::vector<uint32_t>& rbeg = ctx->sbr_rbegin;  // [run + 1] first record of each run
    std::vector<uint32_t>& fmap = ctx->sbr_fmap;    // record -> batch frame
    std::vector<uint32_t>& ups = ctx->sbr_ups;      // upsampled batch frames
    rbeg.assign(b->n_runs + 1, 0);
    fmap.clear();
    ups.clear();
    for (uint32_t r = 0; r < b->n_runs; r++) {
        rbeg[r] = (uint32_t)fmap.size();
        for (uint32_t f = b->frame_begin[r]; f < b->frame_begin[r + 1]; f++) {
            if (frame_dropped(b, f)) continue;  // no record and no PCM (its header: below)
            if (b->sbr[f].status == JAAD_SBR_UPSAMPLE) ups.push_back(f);
            else if (b->sbr[f].status == JAAD_SBR_OK) fmap.push_back(f);
            else {
                ctx->err = "SBR status of frame " + std::to_string(f);
                return JAAD_ERR_INVALID_ARG;
            }
        }
    }
    rbeg[b->n_runs] = (uint32_t)fmap.size();
    const size_t nr = fmap.size(), ncf = nr * nch;  // records, record ch-frames
    const bool identity = nr == nf;  // no upsampled and no dropped frame: record = batch frame

    // chunk plan (records of each run).  Synthesis chunks: one wave each, its 9-slot v history
    // recomputed, a run's records split into chunks of equal length (+-1) of about kSbrSynFrames.
    // (Round 4: chunks sized to fill the resident waves once -- 13 frames on C4 -- ran 10 % slower
    // than 4-frame chunks in 3+ rounds: the synthesis is latency-bound per wave.)
    ctx->sbr_chunks.clear();
    ctx->sbr_last.clear();
    ctx->ps_runs.clear();
    const uint32_t syn_len = std::min<uint32_t>(ctx->syn_frames ? ctx->syn_frames : (uint32_t)kSbrSynFrames, 0xffff);
    for (uint32_t r = 0; r < b->n_runs; r++) {
        const uint32_t i0 = rbeg[r], i1 = rbeg[r + 1];
        if (i1 == i0) continue;  // no SBR frame in this call: the slot's SBR state stays as it is
        const uint32_t len = i1 - i0, parts = (len + syn_len - 1) / syn_len;
        for (int c = 0; c < och; c++)
            for (uint32_t k = 0; k < parts; k++) {
                const uint32_t a = i0 + (uint32_t)((uint64_t)len * k / parts);
                const uint32_t e = i0 + (uint32_t)((uint64_t)len * (k + 1) / parts);
                ctx->sbr_chunks.push_back(SbrChunk{a, (uint16_t)(e - a), (uint8_t)c, 0});
            }
        for (int c = 0; c < nch; c++) ctx->sbr_last.push_back((i1 - 1) * nch + c);
        if (ps) {
            ctx->ps_runs.push_back(i0);
            ctx->ps_runs.push_back(i1 - i0);
        }
    }
    const size_t o_recs = 0, o_psf = al(ncf * sizeof(SbrRec));
    const size_t o_chunks = al(o_psf + (ps ? nr * sizeof(jaad_ps_frame) : 0));
    const size_t o_last = al(o_chunks + ctx->sbr_chunks.size() * sizeof(SbrChunk));
    const size_t o_runs = al(o_last + ctx->sbr_last.size() * sizeof(uint32_t));
    const size_t o_pslist = al(o_runs + ctx->ps_runs.size() * sizeof(uint32_t));
    const size_t o_fix = al(o_pslist + (ps ? nr * sizeof(uint32_t) : 0));
    const size_t o_chains = al(o_fix + ncf * sizeof(uint32_t));
    const size_t o_fmap = al(o_chains + (size_t)b->n_runs * nch * 2 * sizeof(uint32_t));
    const size_t o_ups = al(o_fmap + (identity ? 0 : nr * sizeof(uint32_t)));
    const size_t n1 = al(o_ups + ups.size() * sizeof(uint32_t));

    // JAAD_TRACE_HOST=1: per-call host timings of this stage on stderr (tuning aid)
    static const bool trace = std::getenv("JAAD_TRACE_HOST") != nullptr;
    using clk = std::chrono::steady_clock;
    const auto t_start = clk::now();
    RecSet& S = ctx->rsets[ctx->rset];
    ctx->rset ^= 1;
    if (S.live) HIPCHK(hipEventSynchronize(S.copied));  // its staging may be rewritten
    const auto t_synced = clk::now();
    HIPCHK(S.h1.ensure(n1));
    char* h1 = static_cast<char*>(S.h1.p);
    SbrRec* recs = reinterpret_cast<SbrRec*>(h1 + o_recs);
    jaad_ps_frame* psf = reinterpret_cast<jaad_ps_frame*>(h1 + o_psf);
    if (!ctx->sbr_chunks.empty())
        std::memcpy(h1 + o_chunks, ctx->sbr_chunks.data(), ctx->sbr_chunks.size() * sizeof(SbrChunk));
    if (!ctx->sbr_last.empty())
        std::memcpy(h1 + o_last, ctx->sbr_last.data(), ctx->sbr_last.size() * sizeof(uint32_t));
    if (!identity) std::memcpy(h1 + o_fmap, fmap.data(), nr * sizeof(uint32_t));
    if (!ups.empty()) std::memcpy(h1 + o_ups, ups.data(), ups.size() * sizeof(uint32_t));
    uint32_t* ps_runs_h = reinterpret_cast<uint32_t*>(h1 + o_runs);
    uint32_t* ps_list_h = reinterpret_cast<uint32_t*>(h1 + o_pslist);

    // parameter records: runs are independent streams, so they are built in parallel; each
    // worker owns a contiguous block of runs and writes its E_orig values into its own region
    int nt = ctx->workers ? ctx->workers->size() : 1;
    if (nf < 2048) nt = 1;
    if ((uint32_t)nt > b->n_runs) nt = b->n_runs ? (int)b->n_runs : 1;
    std::vector<uint32_t> rr(nt + 1);
    for (int t = 0; t <= nt; t++) rr[t] = (uint32_t)((uint64_t)b->n_runs * t / nt);
    std::vector<size_t> rbase(nt + 1, 0);  // region offsets in floats
    for (int t = 0; t < nt; t++)
        rbase[t + 1] = rbase[t] + ((size_t)(rbeg[rr[t + 1]] - rbeg[rr[t]]) * nch * SbrHost::kMaxEorig + 63) / 64 * 64;
    const auto& tabs = ctx->sbr_host->tabs();
    const size_t o_tabs = al(rbase[nt] * sizeof(float) + sizeof(float));
    const size_t n2 = o_tabs + SbrHost::kMaxTables * sizeof(SbrTab);
    HIPCHK(S.h2.ensure(n2));
    char* h2 = static_cast<char*>(S.h2.p);
    std::vector<int> rcs(nt, 0), bad(nt, -1);
    std::vector<uint32_t> used(nt, 0);
    std::vector<char> smooth(nt, 0), deps(nt, 0);
    // a failed call must leave every slot's host SBR state as it found it (the device state and
    // the core overlap are untouched then): each run's slot is saved before its first frame
    std::vector<SbrHostSlot> saved(b->n_runs);
    std::vector<char> saved_ok(b->n_runs, 0);
    std::function<void(int)> work = [&](int t) {
        if (t >= nt) return;  // the pool may be wider than this call's run blocks
        float* region = reinterpret_cast<float*>(h2) + rbase[t];
        uint32_t epos = 0;
        uint32_t last_ps = UINT32_MAX;
        bool sm = false, dp = false;
        int kmin = 64, kmax = 0;  // records' band limits of the current run
        for (uint32_t r = rr[t]; r < rr[t + 1] && !rcs[t]; r++) {
            SbrHostSlot& hs = ctx->sbr_slots[b->stream_slot[r]];
            saved[r] = hs;
            saved_ok[r] = 1;
            const uint32_t fe = b->frame_begin[r + 1];
            uint32_t i = rbeg[r];  // record of frame f
            for (uint32_t f = b->frame_begin[r]; f < fe; f++) {
                if (f + 2 < fe)  // the records are large and sparse-read: pull frame f+2 in early
                    for (size_t o = 0; o < sizeof(jaad_sbr_frame); o += 64)
                        __builtin_prefetch(reinterpret_cast<const char*>(&b->sbr[f + 2]) + o);
                const jaad_sbr_frame& F = b->sbr[f];
                // an upsampled frame, and a dropped one whose SBR payload was read before the
                // bitstream ended (SBR.decode ran readHeader / calc_sbr_tables before the
                // EOSException, A/sbr/SBR.java:117-184): the reference still takes its header
                if (F.status == JAAD_SBR_UPSAMPLE || frame_dropped(b, f)) {
                    if (F.header_present) {
                        const int hr = ctx->sbr_host->take_header(hs, F.hdr);
                        if (hr) {
                            rcs[t] = hr;
                            bad[t] = (int)f;
                            break;
                        }
                    }
                    continue;
                }
                if (ps) {
                    if (!ps_frame_ok(F)) {
                        rcs[t] = JAAD_ERR_BITSTREAM;
                        bad[t] = (int)f;
                        break;
                    }
                    if (F.ps_present) psf[i] = F.ps;
                }
                SbrRec* rec = &recs[(size_t)i * nch];
                int rc = ctx->sbr_host->frame(hs, F, nch, i == rbeg[r], b->stream_slot[r], rec, region, epos,
                                              (uint32_t)rbase[t]);
                if (rc) {
                    rcs[t] = rc;
                    bad[t] = (int)f;
                    break;
                }
                if (ps) {  // PS records of the run (the PS kernels walk only these)
                    if (i == rbeg[r]) last_ps = UINT32_MAX;
                    rec->ps_back = 0;
                    if (last_ps != UINT32_MAX) {
                        if (i - last_ps > 0xffffu) {
                            rcs[t] = JAAD_ERR_UNSUPPORTED;  // > 65535 records without PS data in one call
                            bad[t] = (int)f;
                            break;
                        }
                        rec->ps_back = (uint16_t)(i - last_ps);
                    }
                    if (F.ps_present) {
                        rec->flags |= kSbrPsOn;
                        last_ps = i;
                    }
                }
                sm |= (rec[0].flags & kSbrSmooth) != 0;
                for (int c = 0; c < nch; c++) {
                    dp |= (rec[c].flags & kSbrDep) != 0;
                    kmin = std::min<int>(kmin, rec[c].blim);
                    kmax = std::max<int>(kmax, rec[c].blim);
                }
                i++;
            }
            if (rcs[t]) break;
            if (i > rbeg[r])
                for (int c = 0; c < nch; c++) recs[(size_t)(i - 1) * nch + c].flags |= kSbrLast;
            // one band limit for the whole run: the highest of its records' and of the stream's
            // past (a band's PS all-pass state is zero only if no frame ever had input there);
            // rewritten only where a record's own limit is lower
            const int K = std::max(hs.blim_hw, kmax);
            if (kmin < K)
                for (size_t cf = (size_t)rbeg[r] * nch; cf < (size_t)i * nch; cf++) recs[cf].blim = (uint8_t)K;
            hs.blim_hw = K;
            kmin = 64;
            kmax = 0;
        }
        used[t] = epos;
        smooth[t] = sm;
        deps[t] = dp;
    };
    if (nt > 1) ctx->workers->run(work);
    else work(0);
    const auto t_built = clk::now();
    bool smoothing = false, any_dep = false;
    for (int t = 0; t < nt; t++) {
        if (rcs[t]) {
            // restore every run any worker started (a worker stops at its first bad frame)
            for (uint32_t r = 0; r < b->n_runs; r++)
                if (saved_ok[r]) ctx->sbr_slots[b->stream_slot[r]] = saved[r];
            ctx->err = (ps ? "SBR/PS side info of frame " : "SBR side info of frame ") + std::to_string(bad[t]);
            return rcs[t];
        }
        smoothing |= smooth[t] != 0;
        any_dep |= deps[t] != 0;
    }
    if (ps) {  // per run: (offset, count) of its PS records in ps_list
        uint32_t np = 0, ri = 0;
        for (uint32_t r = 0; r < b->n_runs; r++) {
            const uint32_t i0 = rbeg[r], i1 = rbeg[r + 1];
            if (i1 == i0) continue;
            const uint32_t off = np;
            for (uint32_t i = i0; i < i1; i++)
                if (recs[i].flags & kSbrPsOn) ps_list_h[np++] = i;
            ps_runs_h[2 * ri] = off;
            ps_runs_h[2 * ri + 1] = np - off;
            ri++;
        }
    }
    if (!tabs.empty()) std::memcpy(h2 + o_tabs, tabs.data(), tabs.size() * sizeof(SbrTab));

    // HF fix passes: a kSbrDep channel-frame needs frame f-1's final carry rows, so it is
    // recomputed in pass d = its link count down a chain of such frames (with G/Q smoothing a
    // frame whose predecessor was recomputed is recomputed too: its ring came from that frame)
    // Chains longer than kSbrFixPasses (bs_smoothing_mode 0 after a kSbrDep frame can run to the
    // end of the run) are not walked one launch per link: their frames past that depth go to one
    // sequential walker launch, a wave per (run, channel) stepping frame by frame.
    std::vector<uint32_t> fix_counts;
    uint32_t n_chains = 0;
    if (any_dep) {
        uint32_t* fix_h = reinterpret_cast<uint32_t*>(h1 + o_fix);
        uint32_t* chains_h = reinterpret_cast<uint32_t*>(h1 + o_chains);
        std::vector<uint32_t>& depth = ctx->sbr_depth;
        depth.assign(ncf, 0);
        uint32_t max_d = 0;
        for (uint32_t r = 0; r < b->n_runs; r++)
            for (uint32_t i = rbeg[r] + 1; i < rbeg[r + 1]; i++)
                for (int c = 0; c < nch; c++) {
                    const size_t cf = (size_t)i * nch + c;
                    const uint8_t fl = recs[cf].flags;
                    const uint32_t dp = depth[cf - nch];
                    if ((fl & kSbrDep) || ((fl & kSbrSmooth) && !(fl & kSbrReset) && dp > 0)) {
                        depth[cf] = dp + 1;
                        max_d = std::max(max_d, dp + 1);
                    }
                }
        const uint32_t np = std::min<uint32_t>(max_d, kSbrFixPasses);
        fix_counts.assign(np, 0);
        for (size_t cf = 0; cf < ncf; cf++)
            if (depth[cf] && depth[cf] <= np) fix_counts[depth[cf] - 1]++;
        std::vector<uint32_t> pos(np + 1, 0);
        for (uint32_t d = 0; d < np; d++) pos[d + 1] = pos[d] + fix_counts[d];
        for (size_t cf = 0; cf < ncf; cf++)
            if (depth[cf] && depth[cf] <= np) fix_h[pos[depth[cf] - 1]++] = (uint32_t)cf;
        if (max_d > np) {  // the walker's lists follow the passes' (frame order per run and channel)
            uint32_t at = pos[np];
            for (uint32_t r = 0; r < b->n_runs; r++)
                for (int c = 0; c < nch; c++) {
                    const uint32_t o = at;
                    for (uint32_t i = rbeg[r]; i < rbeg[r + 1]; i++) {
                        const size_t cf = (size_t)i * nch + c;
                        if (depth[cf] > np) fix_h[at++] = (uint32_t)cf;
                    }
                    if (at > o) {
                        chains_h[2 * n_chains] = o - pos[np];
                        chains_h[2 * n_chains + 1] = at - o;
                        n_chains++;
                    }
                }
        }
    }
    const auto t_packed = clk::now();

    // device side: intermediates (stream-ordered) and this set's record copy (copy stream)
    HIPCHK(ctx->d_xlow.ensure(ncf * 2048 * sizeof(float) + 256));
    if (!ps) HIPCHK(ctx->d_xsyn.ensure(ncf * 4096 * sizeof(float) + 256));  // (PS: the HF kernel writes into xps)
    HIPCHK(ctx->d_xcarry.ensure(ncf * kSbrCarryFloats * sizeof(float) + 256));
    HIPCHK(ctx->d_gq.ensure(ncf * 640 * sizeof(float) + 256));
    if (ps) {
        HIPCHK(ctx->d_xps.ensure(nr * 8192 * sizeof(float) + 256));
        HIPCHK(ctx->d_xhl.ensure(nr * 768 * sizeof(float) + 256));
        HIPCHK(ctx->d_xhr.ensure(nr * 768 * sizeof(float) + 256));
        HIPCHK(ctx->d_pg.ensure(nr * 640 * sizeof(float) + 256));
        HIPCHK(ctx->d_hb.ensure(nr * 5 * 22 * 16 * sizeof(float) + 256));
    }
    HIPCHK(S.d1.ensure(n1 + 256));
    HIPCHK(S.d2.ensure(n2 + 256));
    // (the launch pipeline queues them on its H2D stream: a third copy stream shared an engine with
    // its D2H copies, and the records of every piece waited for the previous piece's PCM)
    hipStream_t up = ctx->rec_stream ? ctx->rec_stream : ctx->cstream;
    if (S.live) HIPCHK(hipStreamWaitEvent(up, S.used, 0));  // kernels of two calls ago
    HIPCHK(hipMemcpyAsync(S.d1.p, h1, n1, hipMemcpyHostToDevice, up));
    for (int t = 0; t < nt; t++)
        if (used[t])
            HIPCHK(hipMemcpyAsync(static_cast<char*>(S.d2.p) + rbase[t] * sizeof(float), h2 + rbase[t] * sizeof(float),
                                  used[t] * sizeof(float), hipMemcpyHostToDevice, up));
    if (!tabs.empty())
        HIPCHK(hipMemcpyAsync(static_cast<char*>(S.d2.p) + o_tabs, h2 + o_tabs, tabs.size() * sizeof(SbrTab),
                              hipMemcpyHostToDevice, up));
    HIPCHK(hipEventRecord(S.copied, up));
    HIPCHK(hipStreamWaitEvent(stream, S.copied, 0));
    const char* d1 = static_cast<const char*>(S.d1.p);
    const char* d2 = static_cast<const char*>(S.d2.p);

    SbrArgs a{};
    a.time = static_cast<const float*>(ctx->d_time.p);
    a.fmap = identity ? nullptr : reinterpret_cast<const uint32_t*>(d1 + o_fmap);
    a.ups = reinterpret_cast<const uint32_t*>(d1 + o_ups);
    a.n_ups = (uint32_t)ups.size();
    a.recs = reinterpret_cast<const SbrRec*>(d1 + o_recs);
    a.epool = reinterpret_cast<const float*>(d2);
    a.tabs = reinterpret_cast<const SbrTab*>(d2 + o_tabs);
    a.xlow = static_cast<float*>(ctx->d_xlow.p);
    a.xsyn = static_cast<float*>(ctx->d_xsyn.p);
    a.xcarry = static_cast<float*>(ctx->d_xcarry.p);
    a.gq = static_cast<float*>(ctx->d_gq.p);
    a.chunks = reinterpret_cast<const SbrChunk*>(d1 + o_chunks);
    a.last_cf = reinterpret_cast<const uint32_t*>(d1 + o_last);
    a.state = ctx->d_sbr_state;
    a.pcm = pcm;
    a.qmf_c = ctx->d_sbr_const;
    a.dct = ctx->d_sbr_const + 640;
    a.noise = ctx->d_sbr_const + 640 + 224;
    a.down = sbr_downsampled(ctx->cfg) ? 1 : 0;
    a.tw32 = ctx->d_sbr_const + kSbrConstTw32;
    a.n_cf = (uint32_t)ncf;
    a.n_chunks = (uint32_t)ctx->sbr_chunks.size();
    a.n_last = (uint32_t)ctx->sbr_last.size();
    a.nch = nch;
    a.out_mode = flags;
    a.smoothing = smoothing ? 1 : 0;
    a.dbg = ctx->sbr_dbg;
    if (ps) {
        a.ps = 1;
        a.psf = reinterpret_cast<const jaad_ps_frame*>(d1 + o_psf);
        a.psc = ctx->d_ps_const;
        a.zero = ctx->d_ps_zero;
        a.pss = ctx->d_ps_state;
        a.xps = static_cast<float*>(ctx->d_xps.p);
        a.xhl = static_cast<float*>(ctx->d_xhl.p);
        a.xhr = static_cast<float*>(ctx->d_xhr.p);
        a.pg = static_cast<float*>(ctx->d_pg.p);
        a.hb = static_cast<float*>(ctx->d_hb.p);
        a.runs = reinterpret_cast<const uint32_t*>(d1 + o_runs);
        a.ps_list = reinterpret_cast<const uint32_t*>(d1 + o_pslist);
        a.n_runs = (uint32_t)(ctx->ps_runs.size() / 2);
    }
    a.chains = reinterpret_cast<const uint32_t*>(d1 + o_chains);
    a.n_chains = n_chains;
    LAUNCHCHK(launch_sbr(a, stream, reinterpret_cast<const uint32_t*>(d1 + o_fix), fix_counts.data(),
                         (int)fix_counts.size()), stream);
    HIPCHK(hipEventRecord(S.used, stream));
    S.live = true;
    if (trace) {
        auto ms = [](clk::time_point a, clk::time_point b) { return std::chrono::duration<double, std::milli>(b - a).count(); };
        size_t eu = 0;
        for (int t = 0; t < nt; t++) eu += used[t];
        std::fprintf(stderr, "jaad sbr host: wait %.3f build %.3f pack %.3f enqueue %.3f ms (threads %d, %zu+%zu B)\n",
                     ms(t_start, t_synced), ms(t_synced, t_built), ms(t_built, t_packed), ms(t_packed, clk::now()), nt,
                     n1, eu * sizeof(float));
    }
    return JAAD_OK;
}

// Dependent coupling of a batch (jaad_gpu.h jaad_cce_term): the terms' frame ranges, targets and
// band gains go to the device with one copy, cce_term_kernel turns each term into its addend, and
// the LC kernel (mode 2) adds a frame's addends to its target channels after M/S and I/S.
int setup_coupling(jaad_ctx* ctx, const jaad_batch* db, KernelArgs& a, hipStream_t stream)
{
    const uint32_t nt = db->n_cce_terms, nf = db->n_frames;
    auto al = [](size_t x) { return (x + 255) & ~(size_t)255; };
    const size_t o_off = 0, o_meta = al(4 * ((size_t)nf + 1)), o_gain = al(o_meta + 4 * (size_t)nt);
    const size_t o_spec = al(o_gain + 480 * (size_t)nt), total = o_spec + 4096 * (size_t)nt;
    HIPCHK(ctx->d_cce.ensure(total + 256));
    if (ctx->done_live) HIPCHK(hipEventSynchronize(ctx->done));  // the previous call's copy of the image is done
    HIPCHK(ctx->h_cce.ensure(o_spec));
    char* h = static_cast<char*>(ctx->h_cce.p);
    uint32_t* off = reinterpret_cast<uint32_t*>(h + o_off);
    uint32_t* meta = reinterpret_cast<uint32_t*>(h + o_meta);
    float* gain = reinterpret_cast<float*>(h + o_gain);
    // a frame's terms in application order: every BEFORE_TNS term, then every AFTER_TNS term (the
    // two processDependentCoupling passes, A/syntax/CPE.java:172-179), each pass in list order
    uint32_t t = 0, o = 0;
    for (uint32_t f = 0; f <= nf; f++) {  // terms are sorted by frame (check_batch)
        off[f] = o;
        uint32_t e = t;
        while (f < nf && e < nt && db->cce_terms[e].frame == f) e++;
        for (uint32_t point = 0; point < 2; point++)
            for (uint32_t i = t; i < e; i++) {
                const jaad_cce_term& T = db->cce_terms[i];
                if (T.point != point) continue;
                meta[o] = (uint32_t)T.cce | ((uint32_t)T.channel << 16) | ((uint32_t)T.point << 24);
                std::memcpy(gain + (size_t)o * 120, T.gain, 480);
                o++;
            }
        t = e;
    }
    char* d = static_cast<char*>(ctx->d_cce.p);
    HIPCHK(hipMemcpyAsync(d, h, o_spec, hipMemcpyHostToDevice, stream));
    CceArgs c{};
    c.q = db->cce_q;
    c.sf = db->cce_sf;
    c.cb = db->cce_cb;
    c.ics = db->cce_ics;
    c.meta = reinterpret_cast<const uint32_t*>(d + o_meta);
    c.gain = reinterpret_cast<const float*>(d + o_gain);
    c.spec = reinterpret_cast<float*>(d + o_spec);
    c.iq_table = ctx->d_iq;
    c.tables = ctx->d_tables;
    c.gtab = ctx->d_gtab;
    c.n_terms = nt;
    LAUNCHCHK(launch_cce_terms(c, stream), stream);
    a.cce_off = reinterpret_cast<const uint32_t*>(d + o_off);
    a.cce_meta = c.meta;
    a.cce_spec = c.spec;
    a.ch0 = 0;
    a.n_cce_terms = o;
    return JAAD_OK;
}

int launch_mc_sbr(jaad_ctx* ctx, const jaad_batch* db, void* pcm, uint32_t flags, hipStream_t stream);

int launch_work(jaad_ctx* ctx, const jaad_batch* db, void* pcm, uint32_t flags, hipStream_t stream)
{
    if (!ctx->children.empty()) return launch_mc_sbr(ctx, db, pcm, flags, stream);
    jaad_batch vb;  // the kept frames (dropped frames are not planned)
    int rc = keep_map(ctx, db, vb);
    if (rc) return rc;
    rc = plan(ctx, &vb, stream);
    if (rc) return rc;
    KernelArgs a{};
    a.q = db->q;
    a.sf = db->sf;
    a.cb = db->cb;
    a.ics = db->ics;
    a.ms_used = db->ms_used;
    a.tns = db->tns;
    a.iq_table = ctx->d_iq;
    a.tables = ctx->d_tables;
    a.gtab = ctx->d_gtab;
    a.chunks = chunks_dev(ctx);
    a.state_in = ctx->d_state[ctx->parity];
    a.state_out = ctx->d_state[ctx->parity ^ 1];
    const bool sbr = ctx->cfg.sbr != 0;
    if (sbr || ctx->n_elem > 1)
        HIPCHK(ctx->d_time.ensure((size_t)db->n_frames * ctx->nch * 1024 * sizeof(float) + 256));
    a.pcm = sbr ? ctx->d_time.p : pcm;
    a.n_chunks = (uint32_t)ctx->chunks.size();
    a.nch = (uint32_t)ctx->nch;
    a.cf_stride = (uint32_t)ctx->nch;
    a.ms_stride = 1;
    a.out_mode = sbr ? kOutPlanarF32 : flags;
    a.tns_mode = ctx->cfg.tns_mode;
    a.dbg = ctx->dbg;
    a.dbg_frame = ctx->dbg_frame;
    a.skips = plan_skips_dev(ctx);
    a.n_skip_pairs = (uint32_t)(ctx->plan_skips.size() / 2);
    a.frame_lo = 0;
    a.frame_hi = db->n_frames;
    a.n_slots = ctx->n_slots;
    // the fused (+-1 LSB) instantiation serves AAC-LC output only: an SBR context's core samples
    // feed the QMF analysis, whose stages are all kept exact
    a.precision = sbr ? (uint32_t)JAAD_PRECISION_EXACT : ctx->cfg.precision;
    a.short_pair = ctx->hint_short ? 1u : 0u;
    if (a.n_chunks == 0) return JAAD_OK;
    if (db->n_cce_terms && (rc = setup_coupling(ctx, db, a, stream))) return rc;
    if (ctx->n_elem > 1) {
        // Multichannel: each element decodes from its own channel-frame columns (stride = all
        // channels) and its own state region into planar f32 columns; one pack pass then
        // interleaves the channels in element order (SampleBuffer.accept, S/SampleBuffer.java:187-207)
        const bool tns_spec = ctx->cfg.tns_mode == JAAD_TNS_SPEC && db->tns != nullptr;
        int ch0 = 0, cpe = 0;
        for (int k = 0; k < ctx->n_elem; k++) {
            KernelArgs e = a;
            const int n = ctx->elem_nch[k];
            e.q = db->q + (size_t)ch0 * 1024;
            e.sf = db->sf + (size_t)ch0 * 128;
            e.cb = db->cb + (size_t)ch0 * 128;
            e.ics = db->ics + ch0;
            e.tns = db->tns ? db->tns + ch0 : nullptr;
            e.ms_used = n == 2 && db->ms_used ? db->ms_used + 2 * cpe : nullptr;
            e.ms_stride = (uint32_t)ctx->n_cpe;
            e.nch = (uint32_t)n;
            const size_t region = (size_t)k * ctx->n_slots * 2048;
            e.state_in = a.state_in + region;
            e.state_out = a.state_out + region;
            e.pcm = static_cast<float*>(ctx->d_time.p) + (size_t)ch0 * 1024;
            e.out_mode = kOutPlanarF32;
            e.ch0 = (uint32_t)ch0;
            if ((rc = carry_untouched(ctx, e.state_out, e.state_in, 2048, stream))) return rc;
            LAUNCHCHK(launch_lc(e, stream, tns_spec), stream);
            ch0 += n;
            cpe += n == 2;
        }
        LAUNCHCHK(launch_pack(static_cast<const float*>(ctx->d_time.p), pcm, db->n_frames, ctx->nch, flags, stream, a.skips,
                              n_skip_runs(ctx)), stream);
        ctx->parity ^= 1;
        return JAAD_OK;
    }
    rc = carry_untouched(ctx, a.state_out, a.state_in, 2048, stream);
    if (rc) return rc;
    const bool tns_spec = ctx->cfg.tns_mode == JAAD_TNS_SPEC && db->tns != nullptr;
    LAUNCHCHK(launch_lc(a, stream, tns_spec), stream);
    if (sbr && (rc = launch_sbr_stage(ctx, db, pcm, flags, stream))) return rc;
    ctx->parity ^= 1;
    return JAAD_OK;
}

int launch(jaad_ctx* ctx, const jaad_batch* db, void* pcm, uint32_t flags, hipStream_t stream);

// Dry run of launch_sbr_stage's record checks (header tables, mixed tables of a header taken on an
// upsampled or dropped frame, PS parameters) on copies of the slots' host SBR state: nothing of the
// context moves.  A multichannel call runs it for every element before it launches any of them, so
// a rejected batch leaves every element's state as it was.
int sbr_records_ok(jaad_ctx* ctx, const jaad_batch* b)
{
    const int nch = ctx->nch;
    std::vector<SbrRec> rec(nch);
    std::vector<float> pool((size_t)nch * SbrHost::kMaxEorig + 64);
    for (uint32_t r = 0; r < b->n_runs; r++) {
        SbrHostSlot hs = ctx->sbr_slots[b->stream_slot[r]];
        bool first = true;
        for (uint32_t f = b->frame_begin[r]; f < b->frame_begin[r + 1]; f++) {
            const jaad_sbr_frame& F = b->sbr[f];
            if (F.status == JAAD_SBR_UPSAMPLE || frame_dropped(b, f)) {
                if (F.header_present) {
                    const int rc = ctx->sbr_host->take_header(hs, F.hdr);
                    if (rc) return rc;
                }
                continue;
            }
            if (F.status != JAAD_SBR_OK) return JAAD_ERR_INVALID_ARG;
            if (ctx->cfg.ps && !ps_frame_ok(F)) return JAAD_ERR_BITSTREAM;
            uint32_t epos = 0;
            const int rc = ctx->sbr_host->frame(hs, F, nch, first, b->stream_slot[r], rec.data(), pool.data(), epos, 0);
            if (rc) return rc;
            first = false;
        }
    }
    return JAAD_OK;
}

// Multichannel HE-AAC.  Element k's records (its channel columns of q/sf/cb/ics/tns, its ms_used pair,
// its SBR record of each frame) are gathered into contiguous arrays by strided device copies and
// decoded by the element's own SBR context into [frame][sample][2] PCM (an SCE's SBR1 output is
// dataL and its copy dataR, A/sbr/SBR1.java:75-81; a CPE's SBR2 gives L and R; the LFE's records are
// all JAAD_SBR_UPSAMPLE, A/sbr/SBR.java:302-309).  One pass then interleaves the elements' channels
// in element order, as SyntacticElements.process collects them (A/syntax/SyntacticElements.java:
// 235-248): SCE 2, CPE 2, LFE 1 (its left).  Byte order / float32 are already the children's.
int launch_mc_sbr(jaad_ctx* ctx, const jaad_batch* db, void* pcm, uint32_t flags, hipStream_t stream)
{
    const size_t nf = db->n_frames;
    const int ne = ctx->n_elem, nch = ctx->nch;
    if (!db->sbr) return JAAD_ERR_INVALID_ARG;
    jaad_batch vb;  // dropped frames: each child skips them, the interleave pass leaves their PCM
    int krc = keep_map(ctx, db, vb);
    if (krc) return krc;
    const uint32_t* d_skips = nullptr;
    if ((krc = upload_skips(ctx, stream, &d_skips))) return krc;
    const uint32_t n_skips = n_skip_runs(ctx);
    // element kinds of the layout: an SCE must carry SBR data in every frame (without it the
    // reference's channel list shrinks, A/syntax/SCE.java:122-132), an LFE never does
    for (size_t f = 0; f < nf; f++)
        for (int k = 0; k < ne; k++) {
            if (frame_dropped(db, f)) continue;
            const jaad_sbr_frame& r = db->sbr[f * ne + k];
            const bool lfe = mc_is_lfe(ctx->cfg.channel_config, k, ne);
            if (lfe ? r.status != JAAD_SBR_UPSAMPLE : (ctx->elem_nch[k] == 1 && r.status == JAAD_SBR_UPSAMPLE))
                return JAAD_ERR_UNSUPPORTED;
        }
    // every element's SBR records are checked before the first element is launched
    for (int k = 0; k < ne; k++) {
        ctx->h_mc_sbr.resize(nf);
        for (size_t f = 0; f < nf; f++) ctx->h_mc_sbr[f] = db->sbr[f * ne + k];
        jaad_batch c = *db;
        c.sbr = ctx->h_mc_sbr.data();
        const int rc = sbr_records_ok(ctx->children[k], &c);
        if (rc) {
            ctx->err = "SBR side info of element " + std::to_string(k);
            return rc;
        }
    }
    auto al = [](size_t x) { return (x + 255) & ~(size_t)255; };
    const size_t S = (size_t)jaad_cfg_sample_length(&ctx->cfg), bps = (flags & JAAD_PCM_FLOAT32) ? 4 : 2;
    const size_t pcm_k = al(nf * S * 2 * bps);  // one element's PCM
    // per element: q | sf | cb | ics | ms | tns | pcm, each 256-B aligned (sized for a CPE)
    const size_t o_sf = al(nf * 2 * 2048), o_cb = o_sf + al(nf * 2 * 128), o_ics = o_cb + al(nf * 2 * 128);
    const size_t o_ms = o_ics + al(nf * 2 * sizeof(jaad_ics_info)), o_tns = o_ms + al(nf * 16);
    const size_t o_pcm = o_tns + (db->tns ? al(nf * 2 * sizeof(jaad_tns)) : 0), per_el = o_pcm + pcm_k;
    HIPCHK(ctx->d_mc.ensure(per_el * ne + 256));
    char* base = static_cast<char*>(ctx->d_mc.p);
    int ch0 = 0, cpe = 0;
    for (int k = 0; k < ne; k++) {
        const int n = ctx->elem_nch[k];
        char* e = base + per_el * k;
        if (nf) {
            auto gather = [&](size_t off, const void* src, size_t per_ch) {
                return hipMemcpy2DAsync(e + off, n * per_ch, static_cast<const char*>(src) + ch0 * per_ch, nch * per_ch,
                                        n * per_ch, nf, hipMemcpyDeviceToDevice, stream);
            };
            HIPCHK(gather(0, db->q, 2048));
            HIPCHK(gather(o_sf, db->sf, 128));
            HIPCHK(gather(o_cb, db->cb, 128));
            HIPCHK(gather(o_ics, db->ics, sizeof(jaad_ics_info)));
            if (db->tns) HIPCHK(gather(o_tns, db->tns, sizeof(jaad_tns)));
            if (n == 2)
                HIPCHK(hipMemcpy2DAsync(e + o_ms, 16, db->ms_used + 2 * cpe, 16 * (size_t)ctx->n_cpe, 16, nf,
                                        hipMemcpyDeviceToDevice, stream));
        }
        ctx->h_mc_sbr.resize(nf);
        for (size_t f = 0; f < nf; f++) ctx->h_mc_sbr[f] = db->sbr[f * ne + k];
        jaad_batch c{};
        c.n_frames = db->n_frames;
        c.n_runs = db->n_runs;
        c.stream_slot = db->stream_slot;
        c.frame_begin = db->frame_begin;
        c.frame_status = db->frame_status;
        c.q = reinterpret_cast<const int16_t*>(e);
        c.sf = reinterpret_cast<const uint8_t*>(e + o_sf);
        c.cb = reinterpret_cast<const uint8_t*>(e + o_cb);
        c.ics = reinterpret_cast<const jaad_ics_info*>(e + o_ics);
        c.ms_used = n == 2 ? reinterpret_cast<const uint64_t*>(e + o_ms) : nullptr;
        c.tns = db->tns ? reinterpret_cast<const jaad_tns*>(e + o_tns) : nullptr;
        c.sbr = ctx->h_mc_sbr.data();
        // dependent coupling of this element's channels (the CCE records are shared)
        ctx->h_mc_terms.clear();
        for (uint32_t t = 0; t < db->n_cce_terms; t++) {
            const jaad_cce_term& T = db->cce_terms[t];
            if (T.channel < ch0 || T.channel >= ch0 + n) continue;
            ctx->h_mc_terms.push_back(T);
            ctx->h_mc_terms.back().channel = (uint8_t)(T.channel - ch0);
        }
        if (!ctx->h_mc_terms.empty()) {
            c.n_cce = db->n_cce;
            c.cce_q = db->cce_q;
            c.cce_sf = db->cce_sf;
            c.cce_cb = db->cce_cb;
            c.cce_ics = db->cce_ics;
            c.n_cce_terms = (uint32_t)ctx->h_mc_terms.size();
            c.cce_terms = ctx->h_mc_terms.data();
        }
        // the child's SBR records and coupling terms are consumed on the host during this call
        // (launch_sbr_stage, setup_coupling), so h_mc_sbr / h_mc_terms are free again when it returns
        const int rc = launch(ctx->children[k], &c, e + o_pcm, flags, stream);
        if (rc) return rc;
        ch0 += n;
        cpe += n == 2;
    }
    McInterleave m{};
    m.n_out = 0;
    for (int k = 0; k < ne; k++) {
        const int outs = mc_is_lfe(ctx->cfg.channel_config, k, ne) ? 1 : 2;
        for (int j = 0; j < outs; j++) {
            m.src[m.n_out] = base + per_el * k + o_pcm;
            m.chan[m.n_out] = j;
            m.n_out++;
        }
    }
    LAUNCHCHK(launch_mc_interleave(m, pcm, (uint32_t)nf, (uint32_t)S, (int)bps, stream, d_skips, n_skips), stream);
    return JAAD_OK;
}

int launch(jaad_ctx* ctx, const jaad_batch* db, void* pcm, uint32_t flags, hipStream_t stream)
{
    // a call on the stream of the previous call is ordered after it by the stream itself; only a
    // switch of streams needs the wait (an extra barrier packet per call otherwise)
    if (ctx->done_live && stream != ctx->last_stream) HIPCHK(hipStreamWaitEvent(stream, ctx->done, 0));
    const int rc = launch_work(ctx, db, pcm, flags, stream);
    // recorded on failure too: whatever part of the call was queued is covered by the next wait
    HIPCHK(hipEventRecord(ctx->done, stream));
    ctx->done_live = true;
    ctx->last_stream = stream;
    return rc;
}

}  // namespace

extern "C" {

int jaad_cfg_sample_length(const jaad_stream_cfg* cfg)
{
    // frameLengthFlag = 0; doubled by upsampling SBR (A/DecoderConfig.java:83-86)
    return cfg && cfg->sbr && cfg->ext_sf_index != cfg->sf_index ? 2048 : 1024;
}

int jaad_cfg_channel_count(const jaad_stream_cfg* cfg)
{
    // mono is duplicated while sbrEnabled (A/DecoderConfig.java:108-115); configurations 3..7 carry
    // 3, 4, 5, 6 (5.1) and 8 (7.1) channels (ChannelConfiguration, A/ChannelConfiguration.java)
    if (cfg && cfg->channel_config >= 3 && cfg->channel_config <= 7) {
        if (!cfg->sbr) return cfg->channel_config == 7 ? 8 : cfg->channel_config;
        // multichannel HE-AAC: SyntacticElements.process collects dataL and dataR of every SCE with
        // SBR (A/syntax/SCE.java:115-132) and of every CPE, one channel of the LFE (no SBR data,
        // upsampled): configuration 3 -> 4, 4 -> 6, 5 -> 6, 6 -> 7, 7 -> 9
        uint8_t nch[kMaxElements];
        const int n = mc_elements(cfg->channel_config, nch);
        int out = 0;
        for (int k = 0; k < n; k++) out += mc_is_lfe(cfg->channel_config, k, n) ? 1 : 2;
        return out;
    }
    return 2;
}

size_t jaad_frame_pcm_bytes(const jaad_stream_cfg* cfg, uint32_t flags)
{
    return (size_t)jaad_cfg_sample_length(cfg) * jaad_cfg_channel_count(cfg) * ((flags & JAAD_PCM_FLOAT32) ? 4 : 2);
}

const char* jaad_strerror(int status)
{
    switch (status) {
    case JAAD_OK: return "ok";
    case JAAD_ERR_INVALID_ARG: return "invalid argument";
    case JAAD_ERR_NO_DEVICE: return "no usable gfx950 device";
    case JAAD_ERR_HIP: return "HIP runtime error";
    case JAAD_ERR_UNSUPPORTED: return "unsupported configuration";
    case JAAD_ERR_BITSTREAM: return "bitstream side info out of range";
    case JAAD_ERR_NOMEM: return "out of memory";
    case JAAD_ERR_ABI: return "ABI version mismatch";
    case JAAD_ERR_EOS: return "end of bitstream inside a frame";
    default: return "unknown status";
    }
}

const char* jaad_last_error(const jaad_ctx* ctx) { return ctx ? ctx->err.c_str() : ""; }

// internal (not in the public header): device buffer receiving SBR stage dumps
int jaad__sbr_debug_attach(jaad_ctx* ctx, void* dev_buf)
{
    if (!ctx) return JAAD_ERR_INVALID_ARG;
    ctx->sbr_dbg = static_cast<float*>(dev_buf);
    return JAAD_OK;
}

// internal (not in the public header): device buffer of 6144 floats receiving stage dumps
int jaad__debug_attach(jaad_ctx* ctx, void* dev_buf, int frame)
{
    if (!ctx) return JAAD_ERR_INVALID_ARG;
    ctx->dbg = static_cast<float*>(dev_buf);
    ctx->dbg_frame = frame;
    return JAAD_OK;
}

int jaad_ctx_create(const jaad_stream_cfg* cfg, uint32_t n_slots, int device, jaad_ctx** out)
{
    if (!out) return JAAD_ERR_INVALID_ARG;
    *out = nullptr;
    int rc = validate_cfg(cfg);
    if (rc) return rc;
    if (n_slots == 0) return JAAD_ERR_INVALID_ARG;
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev <= device || device < 0) return JAAD_ERR_NO_DEVICE;
    hipDeviceProp_t prop;
    if (hipGetDeviceProperties(&prop, device) != hipSuccess) return JAAD_ERR_NO_DEVICE;
    if (std::strncmp(prop.gcnArchName, "gfx950", 6) != 0) return JAAD_ERR_NO_DEVICE;
    jaad_ctx* ctx = new (std::nothrow) jaad_ctx();
    if (!ctx) return JAAD_ERR_NOMEM;
    ctx->cfg = *cfg;
    ctx->device = device;
    ctx->nch = cfg->channel_config == 2 ? 2 : 1;
    ctx->n_cpe = ctx->nch == 2;
    ctx->elem_nch[0] = (uint8_t)ctx->nch;
    if (const int ne = mc_elements(cfg->channel_config, ctx->elem_nch)) {
        ctx->n_elem = ne;
        ctx->nch = 0;
        ctx->n_cpe = 0;
        for (int k = 0; k < ne; k++) {
            ctx->nch += ctx->elem_nch[k];
            ctx->n_cpe += ctx->elem_nch[k] == 2;
        }
    }
    ctx->n_slots = n_slots;
    ctx->n_cu = prop.multiProcessorCount;
    ctx->slot_used.assign(n_slots, 0);
    if (const char* ev = std::getenv("JAAD_CHUNK_FRAMES")) ctx->chunk_frames = (uint32_t)std::atoi(ev);
    if (const char* ev = std::getenv("JAAD_SBR_PIECES")) ctx->sbr_pieces = (uint32_t)std::atoi(ev);
    if (const char* ev = std::getenv("JAAD_SYN_FRAMES")) ctx->syn_frames = (uint32_t)std::atoi(ev);
    auto bail = [&](hipError_t e, const char* what) {
        std::fprintf(stderr, "jaad_ctx_create: %s: %s\n", what, hipGetErrorString(e));
        jaad_ctx_destroy(ctx);
        return JAAD_ERR_HIP;
    };
    hipError_t e;
    if ((e = hipSetDevice(device)) != hipSuccess) return bail(e, "hipSetDevice");
    if ((e = hipStreamCreateWithFlags(&ctx->stream, hipStreamNonBlocking)) != hipSuccess) return bail(e, "hipStreamCreate");
    if ((e = hipEventCreateWithFlags(&ctx->done, hipEventDisableTiming)) != hipSuccess) return bail(e, "hipEventCreate");
    if ((e = hipEventCreateWithFlags(&ctx->chunks_copied[0], hipEventDisableTiming)) != hipSuccess ||
        (e = hipEventCreateWithFlags(&ctx->chunks_copied[1], hipEventDisableTiming)) != hipSuccess ||
        (e = hipEventCreateWithFlags(&ctx->chunks_read[0], hipEventDisableTiming)) != hipSuccess ||
        (e = hipEventCreateWithFlags(&ctx->chunks_read[1], hipEventDisableTiming)) != hipSuccess)
        return bail(e, "hipEventCreate");
    if ((e = hipEventCreateWithFlags(&ctx->skips_copied, hipEventDisableTiming)) != hipSuccess)
        return bail(e, "hipEventCreate");
    size_t sbytes = (size_t)ctx->n_elem * n_slots * 2048 * sizeof(float);  // [element][slot][2][1024]
    for (int i = 0; i < 2; i++) {
        if ((e = hipMalloc(&ctx->d_state[i], sbytes)) != hipSuccess) return bail(e, "hipMalloc state");
        if ((e = hipMemset(ctx->d_state[i], 0, sbytes)) != hipSuccess) return bail(e, "hipMemset state");
    }
    LdsTables* h = new (std::nothrow) LdsTables;
    GlobalTables gt;
    if (!h) {
        jaad_ctx_destroy(ctx);
        return JAAD_ERR_NOMEM;
    }
    build_lds_tables(cfg->sf_index, h, &gt);
    ctx->lc_waves = (uint32_t)lc_resident_waves_per_cu(cfg->tns_mode == JAAD_TNS_SPEC) * (uint32_t)ctx->n_cu;
    if ((e = hipMalloc(&ctx->d_gtab, sizeof(GlobalTables))) != hipSuccess) { delete h; return bail(e, "hipMalloc gtab"); }
    if ((e = hipMemcpy(ctx->d_gtab, &gt, sizeof(GlobalTables), hipMemcpyHostToDevice)) != hipSuccess) { delete h; return bail(e, "hipMemcpy gtab"); }
    if ((e = hipMalloc(&ctx->d_tables, sizeof(LdsTables))) != hipSuccess) { delete h; return bail(e, "hipMalloc tables"); }
    e = hipMemcpy(ctx->d_tables, h, sizeof(LdsTables), hipMemcpyHostToDevice);
    delete h;
    if (e != hipSuccess) return bail(e, "hipMemcpy tables");
    if ((e = hipMalloc(&ctx->d_iq, sizeof(JAAD_IQ_TABLE))) != hipSuccess) return bail(e, "hipMalloc iq");
    if ((e = hipMemcpy(ctx->d_iq, JAAD_IQ_TABLE, sizeof(JAAD_IQ_TABLE), hipMemcpyHostToDevice)) != hipSuccess)
        return bail(e, "hipMemcpy iq");
    if (cfg->sbr && ctx->n_elem > 1) {
        // multichannel HE-AAC: one SBR context per channel element (ChannelElement owns its SBR,
        // A/syntax/ChannelElement.java:39-74); the LFE too (it is upsampled as SBR.upsample does)
        for (int k = 0; k < ctx->n_elem; k++) {
            jaad_stream_cfg c = *cfg;
            c.channel_config = ctx->elem_nch[k] == 2 ? 2 : 1;
            c.ps = 0;
            jaad_ctx* child = nullptr;
            const int crc = jaad_ctx_create(&c, n_slots, device, &child);
            if (crc) {
                jaad_ctx_destroy(ctx);
                return crc;
            }
            ctx->children.push_back(child);
        }
    } else if (cfg->sbr) {
        ctx->sbr_host.reset(new (std::nothrow) SbrHost(cfg->ext_sf_index));
        if (!ctx->sbr_host) {
            jaad_ctx_destroy(ctx);
            return JAAD_ERR_NOMEM;
        }
        ctx->sbr_slots.resize(n_slots);
        for (auto& hs : ctx->sbr_slots) SbrHost::reset_slot(hs);
        if ((e = hipStreamCreateWithFlags(&ctx->cstream, hipStreamNonBlocking)) != hipSuccess)
            return bail(e, "hipStreamCreate copy");
        {
            ctx->workers.reset(new (std::nothrow) WorkerPool(host_threads()));
        }
        for (RecSet& r : ctx->rsets) {
            if ((e = hipEventCreateWithFlags(&r.copied, hipEventDisableTiming)) != hipSuccess) return bail(e, "hipEventCreate");
            if ((e = hipEventCreateWithFlags(&r.used, hipEventDisableTiming)) != hipSuccess) return bail(e, "hipEventCreate");
        }
        const size_t sb = (size_t)n_slots * 2 * sizeof(SbrChState);
        if ((e = hipMalloc(&ctx->d_sbr_state, sb)) != hipSuccess) return bail(e, "hipMalloc sbr state");
        if ((e = hipMemset(ctx->d_sbr_state, 0, sb)) != hipSuccess) return bail(e, "hipMemset sbr state");
        std::vector<float> k(kSbrConstTw32 + 64);
        std::memcpy(k.data(), JAAD_QMF_C, sizeof(JAAD_QMF_C));
        std::memcpy(k.data() + 640, JAAD_DCT4_64_TAB, sizeof(JAAD_DCT4_64_TAB));
        std::memcpy(k.data() + 640 + 192, JAAD_DCT_W_RE, sizeof(JAAD_DCT_W_RE));
        std::memcpy(k.data() + 640 + 208, JAAD_DCT_W_IM, sizeof(JAAD_DCT_W_IM));
        std::memcpy(k.data() + 640 + 224, JAAD_SBR_NOISE_TABLE, sizeof(JAAD_SBR_NOISE_TABLE));
        // downsampled synthesis: qmf32_pre_twiddle (A/sbr/SynthesisFilterbank32.java:5-38) verbatim
        std::memcpy(k.data() + kSbrConstTw32, JAAD_QMF32_PRE_TWIDDLE, sizeof(JAAD_QMF32_PRE_TWIDDLE));
        if ((e = hipMalloc(&ctx->d_sbr_const, k.size() * sizeof(float))) != hipSuccess) return bail(e, "hipMalloc sbr const");
        if ((e = hipMemcpy(ctx->d_sbr_const, k.data(), k.size() * sizeof(float), hipMemcpyHostToDevice)) != hipSuccess)
            return bail(e, "hipMemcpy sbr const");
    }
    if (cfg->ps) {
        const size_t pb = (size_t)n_slots * sizeof(PsState);
        if ((e = hipMalloc(&ctx->d_ps_state, pb)) != hipSuccess) return bail(e, "hipMalloc ps state");
        if ((e = hipMemset(ctx->d_ps_state, 0, pb)) != hipSuccess) return bail(e, "hipMemset ps state");
        std::unique_ptr<PsConst> k(new (std::nothrow) PsConst);
        if (!k) {
            jaad_ctx_destroy(ctx);
            return JAAD_ERR_NOMEM;
        }
        build_ps_const(k.get());
        const size_t kz = (sizeof(PsConst) + 255) & ~(size_t)255, zb = 32 * 64 * 2 * sizeof(float);
        if ((e = hipMalloc(&ctx->d_ps_const, kz + zb)) != hipSuccess) return bail(e, "hipMalloc ps const");
        ctx->d_ps_zero = reinterpret_cast<float*>(reinterpret_cast<char*>(ctx->d_ps_const) + kz);
        if ((e = hipMemset(ctx->d_ps_zero, 0, zb)) != hipSuccess) return bail(e, "hipMemset ps zero");
        if ((e = hipMemcpy(ctx->d_ps_const, k.get(), sizeof(PsConst), hipMemcpyHostToDevice)) != hipSuccess)
            return bail(e, "hipMemcpy ps const");
    }
    *out = ctx;
    return JAAD_OK;
}

void jaad_ctx_destroy(jaad_ctx* ctx)
{
    if (!ctx) return;
    (void)hipSetDevice(ctx->device);
    if (ctx->done_live) (void)hipEventSynchronize(ctx->done);
    // every stream of the context drained before any buffer is freed (copies of a failed call, the
    // record uploads, the pipelines' D2H copies)
    for (hipStream_t st : {ctx->stream, ctx->cstream, ctx->h2d, ctx->d2h})
        if (st) (void)hipStreamSynchronize(st);
    for (jaad_ctx* c : ctx->children) jaad_ctx_destroy(c);
    ctx->children.clear();
    ctx->d_mc.release();
    for (int i = 0; i < 2; i++)
        if (ctx->d_state[i]) (void)hipFree(ctx->d_state[i]);
    if (ctx->d_tables) (void)hipFree(ctx->d_tables);
    if (ctx->d_gtab) (void)hipFree(ctx->d_gtab);
    if (ctx->d_iq) (void)hipFree(ctx->d_iq);
    if (ctx->d_sbr_state) (void)hipFree(ctx->d_sbr_state);
    if (ctx->d_sbr_const) (void)hipFree(ctx->d_sbr_const);
    if (ctx->d_ps_state) (void)hipFree(ctx->d_ps_state);
    if (ctx->d_ps_const) (void)hipFree(ctx->d_ps_const);
    if (ctx->cstream) (void)hipStreamSynchronize(ctx->cstream);
    for (DevBuf* d : {&ctx->d_time, &ctx->d_xlow, &ctx->d_xsyn, &ctx->d_xcarry, &ctx->d_gq, &ctx->d_xps, &ctx->d_xhl,
                      &ctx->d_xhr, &ctx->d_pg, &ctx->d_hb})
        d->release();
    for (RecSet& r : ctx->rsets) {
        r.h1.release();
        r.h2.release();
        r.d1.release();
        r.d2.release();
        if (r.copied) (void)hipEventDestroy(r.copied);
        if (r.used) (void)hipEventDestroy(r.used);
    }
    if (ctx->cstream) (void)hipStreamDestroy(ctx->cstream);
    for (hipStream_t st : {ctx->h2d, ctx->d2h})
        if (st) {
            (void)hipStreamSynchronize(st);
            (void)hipStreamDestroy(st);
        }
    for (int i = 0; i < kMaxPieces; i++)
        for (hipEvent_t ev : {ctx->ev_in[i], ctx->ev_k[i], ctx->ev_out[i]})
            if (ev) (void)hipEventDestroy(ev);
    for (auto& st : ctx->stage_in) st.release();
    for (auto& st : ctx->stage_out) st.release();
    ctx->d_flag.release();
    ctx->h_flag.release();
    ctx->d_cce.release();
    ctx->h_cce.release();
    for (const auto& r : ctx->pinned) {
        if (r.kind == kPinRegistered) (void)hipHostUnregister(reinterpret_cast<void*>(r.p));
        if (r.kind == kPinOwned) (void)hipHostFree(reinterpret_cast<void*>(r.p));
    }
    ctx->io.reset();
    for (int i = 0; i < 2; i++) {
        ctx->d_chunks[i].release();
        ctx->h_chunks[i].release();
    }
    if (ctx->done) (void)hipEventDestroy(ctx->done);
    for (hipEvent_t ev : ctx->chunks_copied)
        if (ev) (void)hipEventDestroy(ev);
    for (hipEvent_t ev : ctx->chunks_read)
        if (ev) (void)hipEventDestroy(ev);
    if (ctx->skips_copied) (void)hipEventDestroy(ctx->skips_copied);
    ctx->d_skips.release();
    ctx->h_skips.release();
    ctx->d_batch.release();
    ctx->d_pcm.release();
    ctx->d_backup.release();
    if (ctx->stream) (void)hipStreamDestroy(ctx->stream);
    delete ctx;
}

static int check_batch(const jaad_ctx* ctx, const jaad_batch* b, size_t pcm_bytes, uint32_t flags)
{
    if (!ctx || !b) return JAAD_ERR_INVALID_ARG;
    if (b->n_frames && (!b->q || !b->sf || !b->cb || !b->ics)) return JAAD_ERR_INVALID_ARG;
    if (ctx->n_cpe && b->n_frames && !b->ms_used) return JAAD_ERR_INVALID_ARG;
    if (ctx->cfg.sbr && b->n_frames && !b->sbr) return JAAD_ERR_INVALID_ARG;
    if (pcm_bytes < pcm_bytes_per_frame(ctx, flags) * b->n_frames) return JAAD_ERR_INVALID_ARG;
    if (flags & ~(uint32_t)(JAAD_PCM_LITTLE_ENDIAN | JAAD_PCM_FLOAT32)) return JAAD_ERR_INVALID_ARG;
    if (b->n_cce_terms) {  // dependent coupling (jaad_gpu.h); with SBR the core is coupled
        // (spec TNS: kernel mode 3 couples around the filters; a multichannel configuration runs it
        // per channel element, the terms' channels relative to the element, round 6)
        if (!b->cce_terms || !b->n_cce || !b->cce_q || !b->cce_sf || !b->cce_cb || !b->cce_ics) return JAAD_ERR_INVALID_ARG;
        if (b->n_cce > JAAD_CCE_MAX_RECORDS) return JAAD_ERR_UNSUPPORTED;  // jaad_cce_term.cce is 16-bit
        for (uint32_t t = 0; t < b->n_cce_terms; t++) {
            const jaad_cce_term& T = b->cce_terms[t];
            if (T.frame >= b->n_frames || (t && T.frame < b->cce_terms[t - 1].frame)) return JAAD_ERR_INVALID_ARG;
            if (T.channel >= ctx->nch || T.point > 1 || T.cce >= b->n_cce) return JAAD_ERR_INVALID_ARG;
            // non-finite or overflowing gains would carry inf/NaN into the IMDCT and the state
            for (float g : T.gain)
                if (!(std::fabs(g) <= JAAD_CCE_GAIN_MAX)) return JAAD_ERR_UNSUPPORTED;
        }
    }
    return JAAD_OK;
}

// host-side range checks the Java parser would have raised as AACException, over ch-frames
// [c0, c1) (ics/TNS records; |q| separately, fused with its copy)
static bool side_info_ok(const jaad_ctx* ctx, const jaad_batch* b, size_t c0, size_t c1)
{
    const int nl = JAAD_SWB_LONG_WINDOW_COUNT[ctx->cfg.sf_index], ns = JAAD_SWB_SHORT_WINDOW_COUNT[ctx->cfg.sf_index];
    for (size_t i = c0; i < c1; i++) {
        if (b->frame_status && b->frame_status[i / ctx->nch] != JAAD_FRAME_DECODE) continue;  // not read
        const jaad_ics_info& ic = b->ics[i];
        if (ic.window_sequence > 3 || ic.window_shape > 1 || ic.window_shape_prev > 1) return false;
        const int lim = ic.window_sequence == JAAD_EIGHT_SHORT_SEQUENCE ? ns : nl;
        if (ic.max_sfb > lim) return false;  // ICStream.java:137-138 / IndexOutOfBounds
        if (b->tns && (ic.flags & JAAD_ICS_TNS)) {
            const jaad_tns& t = b->tns[i];
            if (t.n_filters > 8) return false;
            for (int f = 0; f < t.n_filters; f++)
                if (t.filt[f].order > 20 || t.filt[f].window > 7) return false;  // TNS.java:56-57
        }
    }
    return true;
}

// |q| <= 8190 (IQ_TABLE has 8191 entries) over n values, copying them to dst on the way (dst may
// be null: check only).  Branch-free inner loop: the compiler vectorises the max.
static bool q_ok_copy(const int16_t* src, int16_t* dst, size_t n)
{
    constexpr size_t B = 4096;
    for (size_t o = 0; o < n; o += B) {
        const size_t m = std::min(B, n - o);
        int bad = 0;
        for (size_t k = 0; k < m; k++) bad |= (src[o + k] > 8190) | (src[o + k] < -8190);
        if (bad) return false;
        if (dst) std::memcpy(dst + o, src + o, m * sizeof(int16_t));
    }
    return true;
}

// q_ok_copy (check only) over the ch-frames [c0, c1) of the batch's kept frames
static bool q_ok_kept(const jaad_ctx* ctx, const jaad_batch* b, size_t c0, size_t c1)
{
    if (!b->frame_status) return q_ok_copy(b->q + c0 * 1024, nullptr, (c1 - c0) * 1024);
    for (size_t i = c0; i < c1;) {
        if (b->frame_status[i / ctx->nch] != JAAD_FRAME_DECODE) {
            i++;
            continue;
        }
        size_t e = i + 1;
        while (e < c1 && b->frame_status[e / ctx->nch] == JAAD_FRAME_DECODE) e++;
        if (!q_ok_copy(b->q + i * 1024, nullptr, (e - i) * 1024)) return false;
        i = e;
    }
    return true;
}

// is [p, p + n) inside a range registered with jaad_host_register?
static bool is_pinned(const jaad_ctx* ctx, const void* p, size_t n)
{
    const uintptr_t a = reinterpret_cast<uintptr_t>(p);
    for (const auto& r : ctx->pinned)
        if (a >= r.p && a + n <= r.p + r.n) return true;
    return false;
}

static int io_setup(jaad_ctx* ctx)
{
    if (ctx->h2d) return JAAD_OK;
    HIPCHK(hipStreamCreateWithFlags(&ctx->h2d, hipStreamNonBlocking));
    HIPCHK(hipStreamCreateWithFlags(&ctx->d2h, hipStreamNonBlocking));
    for (int i = 0; i < kMaxPieces; i++) {
        HIPCHK(hipEventCreateWithFlags(&ctx->ev_in[i], hipEventDisableTiming));
        HIPCHK(hipEventCreateWithFlags(&ctx->ev_k[i], hipEventDisableTiming));
        HIPCHK(hipEventCreateWithFlags(&ctx->ev_out[i], hipEventDisableTiming));
    }
    ctx->io.reset(new (std::nothrow) WorkerPool(host_threads()));
    if (!ctx->io) return JAAD_ERR_NOMEM;
    return JAAD_OK;
}

// Pieces of the batch: run-aligned, balanced by frames (run r goes to the piece whose frame
// interval holds its first frame), as many as kMaxPieces with >= kMinPieceFrames each.
static std::vector<uint32_t> cut_pieces(const jaad_batch* b)
{
    const uint32_t nf = b->n_frames;
    uint32_t P = std::min<uint32_t>(kMaxPieces, std::max<uint32_t>(1, nf / kMinPieceFrames));
    P = std::max<uint32_t>(1, std::min<uint32_t>(P, b->n_runs));
    std::vector<uint32_t> run0{0};  // first run of each piece, then n_runs
    for (uint32_t r = 0; r < b->n_runs; r++) {
        const uint32_t piece = (uint32_t)std::min<uint64_t>((uint64_t)b->frame_begin[r] * P / std::max(nf, 1u), P - 1);
        while (run0.size() <= piece) run0.push_back(r);
    }
    while (run0.size() <= P) run0.push_back(b->n_runs);
    run0.back() = b->n_runs;
    // drop empty pieces
    std::vector<uint32_t> out{0};
    for (size_t i = 1; i < run0.size(); i++)
        if (b->frame_begin[run0[i]] > b->frame_begin[out.back()] || i + 1 == run0.size()) out.push_back(run0[i]);
    out.back() = b->n_runs;
    return out;
}

// The whole SBR path and the fallback: validate, copy in, launch, copy out, one after the other.
static int decode_batch_serial(jaad_ctx* ctx, const jaad_batch* b, void* pcm_out, uint32_t flags)
{
    const size_t nf = b->n_frames, ncf = nf * ctx->nch;
    std::atomic<bool> bad{false};
    const int W = ctx->io->size();
    ctx->io->run([&](int t) {
        const size_t c0 = ncf * t / W, c1 = ncf * (t + 1) / W;
        if (!side_info_ok(ctx, b, c0, c1) || !q_ok_kept(ctx, b, c0, c1)) bad = true;
    });
    if (bad) return JAAD_ERR_BITSTREAM;
    if (b->n_cce_terms) {  // the CCE records get the channel records' checks
        jaad_batch cb = *b;
        cb.ics = b->cce_ics;
        cb.tns = nullptr;
        if (!side_info_ok(ctx, &cb, 0, b->n_cce) || !q_ok_copy(b->cce_q, nullptr, (size_t)b->n_cce * 1024))
            return JAAD_ERR_BITSTREAM;
    }
    // one staging allocation, 256-B aligned sub-buffers
    auto al = [](size_t x) { return (x + 255) & ~(size_t)255; };
    size_t o_q = 0, o_sf = al(o_q + ncf * 2048), o_cb = al(o_sf + ncf * 128), o_ics = al(o_cb + ncf * 128);
    const size_t ms_bytes = nf * 16 * (size_t)std::max(ctx->n_cpe, 1);
    size_t o_ms = al(o_ics + ncf * sizeof(jaad_ics_info)), o_tns = al(o_ms + ms_bytes);
    const size_t nce = b->n_cce_terms ? b->n_cce : 0;  // CCE records (coupling batches)
    size_t o_cq = al(o_tns + (b->tns ? ncf * sizeof(jaad_tns) : 0)), o_csf = al(o_cq + nce * 2048);
    size_t o_ccb = al(o_csf + nce * 128), o_cics = al(o_ccb + nce * 128);
    size_t total = al(o_cics + nce * sizeof(jaad_ics_info));
    HIPCHK(ctx->d_batch.ensure(total + 256));
    size_t pbytes = pcm_bytes_per_frame(ctx, flags) * nf;
    HIPCHK(ctx->d_pcm.ensure(pbytes + 256));
    char* base = static_cast<char*>(ctx->d_batch.p);
    hipStream_t s = ctx->stream;
    if (nf) {
        HIPCHK(hipMemcpyAsync(base + o_q, b->q, ncf * 2048, hipMemcpyHostToDevice, s));
        HIPCHK(hipMemcpyAsync(base + o_sf, b->sf, ncf * 128, hipMemcpyHostToDevice, s));
        HIPCHK(hipMemcpyAsync(base + o_cb, b->cb, ncf * 128, hipMemcpyHostToDevice, s));
        HIPCHK(hipMemcpyAsync(base + o_ics, b->ics, ncf * sizeof(jaad_ics_info), hipMemcpyHostToDevice, s));
        if (b->ms_used) HIPCHK(hipMemcpyAsync(base + o_ms, b->ms_used, ms_bytes, hipMemcpyHostToDevice, s));
        if (b->tns) HIPCHK(hipMemcpyAsync(base + o_tns, b->tns, ncf * sizeof(jaad_tns), hipMemcpyHostToDevice, s));
        if (nce) {
            HIPCHK(hipMemcpyAsync(base + o_cq, b->cce_q, nce * 2048, hipMemcpyHostToDevice, s));
            HIPCHK(hipMemcpyAsync(base + o_csf, b->cce_sf, nce * 128, hipMemcpyHostToDevice, s));
            HIPCHK(hipMemcpyAsync(base + o_ccb, b->cce_cb, nce * 128, hipMemcpyHostToDevice, s));
            HIPCHK(hipMemcpyAsync(base + o_cics, b->cce_ics, nce * sizeof(jaad_ics_info), hipMemcpyHostToDevice, s));
        }
    }
    jaad_batch db = *b;
    db.q = reinterpret_cast<const int16_t*>(base + o_q);
    db.sf = reinterpret_cast<const uint8_t*>(base + o_sf);
    db.cb = reinterpret_cast<const uint8_t*>(base + o_cb);
    db.ics = reinterpret_cast<const jaad_ics_info*>(base + o_ics);
    db.ms_used = b->ms_used ? reinterpret_cast<const uint64_t*>(base + o_ms) : nullptr;
    db.tns = b->tns ? reinterpret_cast<const jaad_tns*>(base + o_tns) : nullptr;
    if (nce) {
        db.cce_q = reinterpret_cast<const int16_t*>(base + o_cq);
        db.cce_sf = reinterpret_cast<const uint8_t*>(base + o_csf);
        db.cce_cb = reinterpret_cast<const uint8_t*>(base + o_ccb);
        db.cce_ics = reinterpret_cast<const jaad_ics_info*>(base + o_cics);
    }
    int rc = launch(ctx, &db, ctx->d_pcm.p, flags, s);
    if (rc) return rc;
    // the slots of dropped frames keep what the caller's buffer holds: the copy back covers the
    // whole batch, so they are saved before it and restored after it
    std::vector<uint8_t> kept_pcm;
    const size_t per = pcm_bytes_per_frame(ctx, flags);
    if (b->frame_status)
        for (size_t f = 0; f < nf; f++)
            if (b->frame_status[f] != JAAD_FRAME_DECODE)
                kept_pcm.insert(kept_pcm.end(), static_cast<uint8_t*>(pcm_out) + f * per,
                                static_cast<uint8_t*>(pcm_out) + (f + 1) * per);
    if (nf) HIPCHK(hipMemcpyAsync(pcm_out, ctx->d_pcm.p, pbytes, hipMemcpyDeviceToHost, s));
    HIPCHK(hipStreamSynchronize(s));
    if (!kept_pcm.empty())
        for (size_t f = 0, k = 0; f < nf; f++)
            if (b->frame_status[f] != JAAD_FRAME_DECODE) {
                std::memcpy(static_cast<uint8_t*>(pcm_out) + f * per, kept_pcm.data() + k * per, per);
                k++;
            }
    return JAAD_OK;
}

// AAC-LC: the pieces pipeline.  Every piece's kernels read the call's input state buffer and
// write the output one (pieces touch disjoint slots), so the state flips once, at the end, and a
// piece that fails validation leaves every slot's state as it was before the call.
//
// Per piece two H2D copies: its q (straight from registered caller memory, else from staging) and
// one block with its side info, which the workers pack into staging while they check it (sf, cb,
// ics, ms_used, tns of the piece back to back; four small copies per piece cost ~0.5 ms of DMA
// set-up per C2 batch).  The piece's kernel gets pointers into its block, offset by the piece's
// first channel-frame so that the batch-wide indices land in it.
static int decode_batch_pieces_impl(jaad_ctx* ctx, const jaad_batch* b, void* pcm_out, uint32_t flags,
                                    const std::vector<uint32_t>& run0);

// Every exit waits for the copies and kernels already queued: they read and write caller memory
// (registered buffers are copied by DMA directly), which the caller may free once this returns.
static int decode_batch_pieces(jaad_ctx* ctx, const jaad_batch* b, void* pcm_out, uint32_t flags,
                               const std::vector<uint32_t>& run0)
{
    const int rc = decode_batch_pieces_impl(ctx, b, pcm_out, flags, run0);
    if (rc) {
        for (hipStream_t st : {ctx->h2d, ctx->d2h, ctx->stream})
            if (st) (void)hipStreamSynchronize(st);
        (void)hipGetLastError();
    }
    return rc;
}

static int decode_batch_pieces_impl(jaad_ctx* ctx, const jaad_batch* b, void* pcm_out, uint32_t flags,
                                    const std::vector<uint32_t>& run0)
{
    const int nch = ctx->nch;
    const size_t nf = b->n_frames, ncf = nf * nch;
    const int P = (int)run0.size() - 1;
    const size_t fbytes = pcm_bytes_per_frame(ctx, flags);
    auto al = [](size_t x) { return (x + 255) & ~(size_t)255; };

    // piece frame ranges and the largest piece (chunk sizing, staging)
    std::vector<size_t> F(P + 1);
    size_t maxf = 0;
    for (int i = 0; i <= P; i++) F[i] = b->frame_begin[run0[i]];
    for (int i = 0; i < P; i++) maxf = std::max(maxf, F[i + 1] - F[i]);
    // side block of a piece of nfi frames: [sf][cb][ics][ms_used][tns], 256-B aligned parts
    struct SideLayout {
        size_t sf, cb, ics, ms, tns, bytes;
    };
    auto side_layout = [&](size_t nfi) {
        const size_t nci = nfi * nch;
        SideLayout L;
        L.sf = 0;
        L.cb = al(nci * 128);
        L.ics = L.cb + al(nci * 128);
        L.ms = L.ics + al(nci * sizeof(jaad_ics_info));
        L.tns = L.ms + (b->ms_used ? al(nfi * 16) : 0);
        L.bytes = L.tns + (b->tns ? al(nci * sizeof(jaad_tns)) : 0);
        return L;
    };
    // device image: q batch-wide (the check kernel reads it), then the pieces' side blocks
    std::vector<size_t> SB(P + 1);
    SB[0] = al(ncf * 2048);
    for (int i = 0; i < P; i++) SB[i + 1] = SB[i] + side_layout(F[i + 1] - F[i]).bytes;
    HIPCHK(ctx->d_batch.ensure(SB[P] + 256));
    HIPCHK(ctx->d_pcm.ensure(fbytes * nf + 256));
    char* base = static_cast<char*>(ctx->d_batch.p);
    char* dpcm = static_cast<char*>(ctx->d_pcm.p);
    const int16_t* dq = reinterpret_cast<const int16_t*>(base);

    hipStream_t s = ctx->stream;
    if (ctx->done_live && ctx->last_stream != s) HIPCHK(hipStreamWaitEvent(s, ctx->done, 0));
    {   // the planner reads only the run layout and the frame count (no frame is dropped here)
        jaad_batch db = *b;
        ctx->skips.clear();
        int rc = plan(ctx, &db, s, (uint32_t)maxf);
        if (rc) return rc;
    }
    // chunk range of each piece (chunks are in run order, frames ascending)
    std::vector<uint32_t> C(P + 1);
    for (int i = 0; i <= P; i++) {
        if (i == P) {
            C[i] = (uint32_t)ctx->chunks.size();
            break;
        }
        C[i] = (uint32_t)(std::lower_bound(ctx->chunks.begin(), ctx->chunks.end(), (uint32_t)F[i],
                                           [](const ChunkDesc& c, uint32_t f) { return c.frame0 < f; }) -
                          ctx->chunks.begin());
    }
    KernelArgs a{};
    a.q = dq;
    a.iq_table = ctx->d_iq;
    a.tables = ctx->d_tables;
    a.gtab = ctx->d_gtab;
    a.state_in = ctx->d_state[ctx->parity];
    a.state_out = ctx->d_state[ctx->parity ^ 1];
    a.pcm = dpcm;
    a.nch = (uint32_t)nch;
    a.cf_stride = (uint32_t)nch;
    a.ms_stride = 1;
    a.out_mode = flags;
    a.tns_mode = ctx->cfg.tns_mode;
    a.dbg = ctx->dbg;
    a.dbg_frame = ctx->dbg_frame;
    a.n_slots = ctx->n_slots;
    a.precision = ctx->cfg.precision;
    a.short_pair = ctx->hint_short ? 1u : 0u;
    const bool tns_spec = ctx->cfg.tns_mode == JAAD_TNS_SPEC && b->tns != nullptr;
    int rc;
    if ((rc = carry_untouched(ctx, a.state_out, a.state_in, 2048, s))) return rc;

    // q and PCM: DMA straight from / to registered memory, else through the staging slots
    const bool pin_q = is_pinned(ctx, b->q, ncf * 2048), pin_out = is_pinned(ctx, pcm_out, fbytes * nf);
    const size_t s_side = pin_q ? 0 : al(maxf * nch * 2048);
    for (auto& st : ctx->stage_in) HIPCHK(st.ensure(s_side + side_layout(maxf).bytes));
    if (!pin_out)
        for (auto& st : ctx->stage_out) HIPCHK(st.ensure(maxf * fbytes));

    // |q| <= 8190 is checked on the device, piece by piece, before the piece's kernel (the host never
    // reads q: a registered q goes straight from the caller's memory to HBM); the LC kernel clamps
    // |q| anyway, so a bad piece decodes garbage but touches nothing outside its buffers, and the
    // flag read at the end turns the call into JAAD_ERR_BITSTREAM with the state not flipped
    HIPCHK(ctx->d_flag.ensure(256));
    HIPCHK(ctx->h_flag.ensure(16));
    int* const dflag = static_cast<int*>(ctx->d_flag.p);
    HIPCHK(hipMemsetAsync(dflag, 0, sizeof(int), s));
    WorkerPool& io = *ctx->io;
    const int W = io.size();
    std::atomic<bool> bad{false};
    int queued = 0;  // pieces whose kernels and D2H copies are queued
    auto copy_out = [&](int i) -> int {  // staging -> caller PCM of piece i
        HIPCHK(hipEventSynchronize(ctx->ev_out[i]));
        const char* src = static_cast<const char*>(ctx->stage_out[i % kStageSlots].p);
        char* dst = static_cast<char*>(pcm_out) + F[i] * fbytes;
        const size_t n = (F[i + 1] - F[i]) * fbytes;
        io.run([&](int t) { std::memcpy(dst + n * t / W, src + n * t / W, n * (t + 1) / W - n * t / W); });
        return JAAD_OK;
    };
    // piece i: check its side info and pack it (and q, unless registered) into staging slot i % 2,
    // then queue its two H2D copies on the one H2D copy stream (a second H2D stream shared a DMA
    // engine with the D2H stream and serialised them: C2 e2e 9.4e6 -> 6.5e6 frames/s,
    // profiles/round3_e2e_*); ev_in[i] marks both done
    auto stage_piece = [&](int i) -> int {
        const size_t f0 = F[i], nfi = F[i + 1] - f0, c0 = f0 * nch, nci = nfi * nch;
        const SideLayout L = side_layout(nfi);
        if (i >= kStageSlots)  // the slot's previous piece has been copied
            HIPCHK(hipEventSynchronize(ctx->ev_in[i - kStageSlots]));
        char* st = static_cast<char*>(ctx->stage_in[i % kStageSlots].p);
        char* sd = st + s_side;
        io.run([&](int t) {
            const size_t a0 = nci * t / W, a1 = nci * (t + 1) / W;
            if (!side_info_ok(ctx, b, c0 + a0, c0 + a1)) bad = true;
            if (!pin_q)
                std::memcpy(reinterpret_cast<int16_t*>(st) + a0 * 1024, b->q + (c0 + a0) * 1024,
                            (a1 - a0) * 1024 * sizeof(int16_t));
            std::memcpy(sd + L.sf + a0 * 128, b->sf + (c0 + a0) * 128, (a1 - a0) * 128);
            std::memcpy(sd + L.cb + a0 * 128, b->cb + (c0 + a0) * 128, (a1 - a0) * 128);
            std::memcpy(sd + L.ics + a0 * sizeof(jaad_ics_info), b->ics + c0 + a0, (a1 - a0) * sizeof(jaad_ics_info));
            if (b->tns) std::memcpy(sd + L.tns + a0 * sizeof(jaad_tns), b->tns + c0 + a0, (a1 - a0) * sizeof(jaad_tns));
            if (b->ms_used && t == 0) std::memcpy(sd + L.ms, b->ms_used + f0 * 2, nfi * 16);
        });
        if (bad) return JAAD_OK;
        hipStream_t h = ctx->h2d;
        HIPCHK(hipMemcpyAsync(base + c0 * 2048, pin_q ? (const void*)(b->q + c0 * 1024) : (const void*)st, nci * 2048,
                              hipMemcpyHostToDevice, h));
        HIPCHK(hipMemcpyAsync(base + SB[i], sd, L.bytes, hipMemcpyHostToDevice, h));
        HIPCHK(hipEventRecord(ctx->ev_in[i], h));
        return JAAD_OK;
    };
    // piece i+1 is checked, packed and its copies queued before piece i's kernel: the host work of
    // one piece overlaps the copies of the previous one, and copies stay one piece ahead (copies
    // are served in submission order, so queueing every H2D first would hold the D2H copies back)
    if ((rc = stage_piece(0))) return rc;
    for (int i = 0; i < P && !bad; i++) {
        if (i + 1 < P && (rc = stage_piece(i + 1))) return rc;
        if (bad) break;
        const size_t f0 = F[i], nfi = F[i + 1] - f0, c0 = f0 * nch, nci = nfi * nch;
        const SideLayout L = side_layout(nfi);
        char* sd = base + SB[i];
        a.sf = reinterpret_cast<const uint8_t*>(sd + L.sf) - c0 * 128;
        a.cb = reinterpret_cast<const uint8_t*>(sd + L.cb) - c0 * 128;
        a.ics = reinterpret_cast<const jaad_ics_info*>(sd + L.ics) - c0;
        a.ms_used = b->ms_used ? reinterpret_cast<const uint64_t*>(sd + L.ms) - f0 * 2 : nullptr;
        a.tns = b->tns ? reinterpret_cast<const jaad_tns*>(sd + L.tns) - c0 : nullptr;
        HIPCHK(hipStreamWaitEvent(s, ctx->ev_in[i], 0));
        LAUNCHCHK(launch_check_q(dq + c0 * 1024, nci * 1024, dflag, s), s);
        a.chunks = chunks_dev(ctx) + C[i];
        a.n_chunks = C[i + 1] - C[i];
        a.frame_lo = (uint32_t)f0;  // the piece's rows: its side block, q and PCM ranges
        a.frame_hi = (uint32_t)(f0 + nfi);
        if (a.n_chunks) LAUNCHCHK(launch_lc(a, s, tns_spec), s);
        HIPCHK(hipEventRecord(ctx->ev_k[i], s));
        HIPCHK(hipStreamWaitEvent(ctx->d2h, ctx->ev_k[i], 0));
        void* dst = pin_out ? static_cast<char*>(pcm_out) + f0 * fbytes : ctx->stage_out[i % kStageSlots].p;
        if (i >= kStageSlots && !pin_out && (rc = copy_out(i - kStageSlots))) return rc;
        HIPCHK(hipMemcpyAsync(dst, dpcm + f0 * fbytes, nfi * fbytes, hipMemcpyDeviceToHost, ctx->d2h));
        HIPCHK(hipEventRecord(ctx->ev_out[i], ctx->d2h));
        queued = i + 1;
    }
    if (!pin_out)
        for (int i = std::max(0, queued - kStageSlots); i < queued; i++)
            if ((rc = copy_out(i))) return rc;
    int* const hflag = static_cast<int*>(ctx->h_flag.p);
    HIPCHK(hipMemcpyAsync(hflag, dflag, sizeof(int), hipMemcpyDeviceToHost, s));
    HIPCHK(hipStreamSynchronize(ctx->d2h));
    HIPCHK(hipStreamSynchronize(ctx->h2d));
    HIPCHK(hipStreamSynchronize(s));
    HIPCHK(hipEventRecord(ctx->done, s));
    ctx->done_live = true;
    ctx->last_stream = s;
    if (bad || *hflag) return JAAD_ERR_BITSTREAM;  // state not flipped: every slot as before the call
    ctx->parity ^= 1;
    return JAAD_OK;
}

// HE-AAC (SBR / PS) and AAC-LC batches with dropped frames: the pieces pipeline through launch().
// Each piece is gathered into a batch of its own and decoded exactly as a call of its own would be
// (LC kernel, SBR records and kernels).  Two ways to cut the batch:
//  * run0 given: run-aligned pieces (whole runs, as the AAC-LC pipeline): a piece is one contiguous
//    range of the caller's arrays, so registered memory goes by plain DMA both ways, and the H2D and
//    D2H copies run on their two engines at once;
//  * run0 null (PS): piece i is the i-th time slice of every run (run r's frames
//    [fb_r + len_r i / P, fb_r + len_r (i+1) / P)), i.e. the i-th of P consecutive calls: the PS
//    decorrelator walks a run's frames in order, so a run-aligned piece would cost a whole run's walk
//    (0.6 ms on C5) however few runs it holds; a slice costs 1/P of it.  The PCM of a slice is R rows
//    of the caller's buffer (a strided D2H copy into registered memory; that copy measured as sharing
//    one engine with the H2D copies, profiles/round5_pipeline/).
// Piece i+1's gather
// (with the host checks: side info, |q|) and H2D copy overlap piece i's kernels and piece i-1's D2H
// copy and scatter.  The call stays all-or-nothing: the core overlap, SBR and PS state of every slot
// are copied aside on the device when it starts (a few us), the host SBR slots on the host, and a
// piece that fails a check or whose SBR records are refused puts them all back.  (The reference
// decodes frame by frame, A/Decoder.java:103-121; multichannel and coupling batches keep the serial
// path.)
// The device state of every slot of a context (and of its elements' child contexts: multichannel
// HE-AAC), copied aside before the first piece's kernels so that a failing piece rolls the whole call
// back: core overlap (the current parity), SBR and PS slot state, and the host-side SBR slot records.
struct StateSnap {
    jaad_ctx* c;
    int parity;
    size_t lc_b, sbr_b, ps_b, off;  // bytes of each part; offset of the context's parts in d_backup
    std::vector<SbrHostSlot> host;
};
static std::vector<StateSnap> state_snaps(jaad_ctx* ctx)
{
    auto al = [](size_t x) { return (x + 255) & ~(size_t)255; };
    std::vector<StateSnap> v;
    size_t off = 0;
    auto add = [&](jaad_ctx* c) {
        // (a multichannel HE-AAC parent holds no SBR state of its own: its children do)
        StateSnap S{c, c->parity, c->d_state[c->parity] ? (size_t)c->n_elem * c->n_slots * 2048 * sizeof(float) : 0,
                    c->cfg.sbr && c->d_sbr_state ? (size_t)c->n_slots * 2 * sizeof(SbrChState) : 0,
                    c->cfg.ps && c->d_ps_state ? (size_t)c->n_slots * sizeof(PsState) : 0, off, {}};
        off += al(S.lc_b) + al(S.sbr_b) + al(S.ps_b);
        v.push_back(std::move(S));
    };
    add(ctx);
    for (jaad_ctx* c : ctx->children) add(c);
    return v;
}

static int decode_batch_pieces_launch_impl(jaad_ctx* ctx, const jaad_batch* b, void* pcm_out, uint32_t flags, int P,
                                           const std::vector<uint32_t>* run0, std::vector<StateSnap>& snaps,
                                           bool& saved)
{
    const int nch = ctx->nch;
    const uint32_t R = b->n_runs;
    const size_t fbytes = pcm_bytes_per_frame(ctx, flags);
    auto al = [](size_t x) { return (x + 255) & ~(size_t)255; };
    auto cut = [&](uint32_t r, int i) {  // first batch frame of run r in pieces >= i
        if (run0) return r < (*run0)[i] ? b->frame_begin[r + 1] : b->frame_begin[r];
        const uint64_t len = b->frame_begin[r + 1] - b->frame_begin[r];
        return b->frame_begin[r] + (uint32_t)(len * (uint64_t)i / (uint64_t)P);
    };
    // per frame: ms_used words (a pair per CPE element) and SBR records (one per channel element)
    const size_t mw = 2 * (size_t)std::max(ctx->n_cpe, 1), sw = (size_t)std::max(ctx->n_elem, 1);
    std::vector<size_t> NF(P + 1, 0);  // first frame of each piece in the pieces' concatenation
    for (int i = 0; i < P; i++) {
        size_t n = 0;
        for (uint32_t r = 0; r < R; r++) n += cut(r, i + 1) - cut(r, i);
        NF[i + 1] = NF[i] + n;
    }
    size_t maxf = 0;
    for (int i = 0; i < P; i++) maxf = std::max(maxf, NF[i + 1] - NF[i]);
    struct Layout {
        size_t q, sf, cb, ics, ms, tns, bytes;
    };
    auto layout = [&](size_t nfi) {
        const size_t nci = nfi * nch;
        Layout L;
        L.q = 0;
        L.sf = al(nci * 2048);
        L.cb = L.sf + al(nci * 128);
        L.ics = L.cb + al(nci * 128);
        L.ms = L.ics + al(nci * sizeof(jaad_ics_info));
        L.tns = L.ms + (b->ms_used ? al(nfi * 8 * mw) : 0);
        L.bytes = L.tns + (b->tns ? al(nci * sizeof(jaad_tns)) : 0);
        return L;
    };
    std::vector<size_t> SB(P + 1, 0);  // device input block of each piece
    for (int i = 0; i < P; i++) SB[i + 1] = SB[i] + layout(NF[i + 1] - NF[i]).bytes;
    // coupling batches: the CCE records once, after the pieces' blocks; each piece gets its frames'
    // terms, renumbered to the piece
    const size_t nce = b->n_cce_terms ? b->n_cce : 0;
    const size_t o_cq = al(SB[P]), o_csf = al(o_cq + nce * 2048), o_ccb = al(o_csf + nce * 128);
    const size_t o_cics = al(o_ccb + nce * 128), in_bytes = al(o_cics + nce * sizeof(jaad_ics_info));
    HIPCHK(ctx->d_batch.ensure(in_bytes + 256));
    HIPCHK(ctx->d_pcm.ensure(fbytes * NF[P] + 256));
    char* base = static_cast<char*>(ctx->d_batch.p);
    char* dpcm = static_cast<char*>(ctx->d_pcm.p);
    hipStream_t s = ctx->stream;
    if (ctx->done_live && ctx->last_stream != s) HIPCHK(hipStreamWaitEvent(s, ctx->done, 0));

    // roll-back copies, queued ahead of every kernel of the call
    snaps = state_snaps(ctx);
    HIPCHK(ctx->d_backup.ensure(snaps.back().off + al(snaps.back().lc_b) + al(snaps.back().sbr_b) + snaps.back().ps_b + 256));
    char* bk = static_cast<char*>(ctx->d_backup.p);
    for (StateSnap& S : snaps) {
        char* o = bk + S.off;
        if (S.lc_b) HIPCHK(hipMemcpyAsync(o, S.c->d_state[S.parity], S.lc_b, hipMemcpyDeviceToDevice, s));
        if (S.sbr_b) HIPCHK(hipMemcpyAsync(o + al(S.lc_b), S.c->d_sbr_state, S.sbr_b, hipMemcpyDeviceToDevice, s));
        if (S.ps_b) HIPCHK(hipMemcpyAsync(o + al(S.lc_b) + al(S.sbr_b), S.c->d_ps_state, S.ps_b, hipMemcpyDeviceToDevice, s));
        S.host = S.c->sbr_slots;
    }
    saved = true;

    // Runs of one length L laid out back to back (the usual batch): a piece is then R rows of one
    // slice length, so registered caller memory is copied by strided DMA straight from / to its
    // place (hipMemcpy2DAsync), no host gather of q or scatter of PCM
    const uint32_t L0 = R ? b->frame_begin[1] - b->frame_begin[0] : 0;
    bool uniform = R > 0;
    for (uint32_t r = 0; r <= R && uniform; r++) uniform = b->frame_begin[r] == r * L0;
    const size_t ncf = (size_t)b->n_frames * nch;
    // Run-aligned pieces: registered q and PCM by plain DMA.  Time slices: q gathered by the workers
    // as they check it (a strided H2D copy measured as sharing one engine with the strided D2H
    // copies: piece i+1's inputs waited for piece i's PCM), PCM by strided DMA when the runs are
    // uniform.
    const bool dma_q = run0 && is_pinned(ctx, b->q, ncf * 2048);
    const bool dma_out = (run0 || uniform) && !b->frame_status && is_pinned(ctx, pcm_out, fbytes * b->n_frames);
    for (auto& st : ctx->stage_in) HIPCHK(st.ensure(layout(maxf).bytes));
    if (!dma_out)
        for (auto& st : ctx->stage_out) HIPCHK(st.ensure(maxf * fbytes));
    WorkerPool& io = *ctx->io;
    const int W = io.size();
    std::atomic<bool> bad{false};
    auto kept = [&](size_t f) { return !b->frame_status || b->frame_status[f] == JAAD_FRAME_DECODE; };
    // the piece's host-side arrays (read by launch() before it returns, so one set serves every piece)
    std::vector<uint32_t> pslot, pbeg, prun;  // runs with frames in the piece: slot, first frame, batch run
    std::vector<jaad_sbr_frame> psbr;
    std::vector<uint8_t> pstat;
    std::vector<jaad_cce_term> pterms;
    if (nce) {  // the CCE records get the channel records' checks (as decode_batch_serial), then one copy
        jaad_batch cb = *b;
        cb.ics = b->cce_ics;
        cb.tns = nullptr;
        if (!side_info_ok(ctx, &cb, 0, b->n_cce) || !q_ok_copy(b->cce_q, nullptr, nce * 1024)) return JAAD_ERR_BITSTREAM;
        HIPCHK(hipMemcpyAsync(base + o_cq, b->cce_q, nce * 2048, hipMemcpyHostToDevice, ctx->h2d));
        HIPCHK(hipMemcpyAsync(base + o_csf, b->cce_sf, nce * 128, hipMemcpyHostToDevice, ctx->h2d));
        HIPCHK(hipMemcpyAsync(base + o_ccb, b->cce_cb, nce * 128, hipMemcpyHostToDevice, ctx->h2d));
        HIPCHK(hipMemcpyAsync(base + o_cics, b->cce_ics, nce * sizeof(jaad_ics_info), hipMemcpyHostToDevice, ctx->h2d));
    }
    auto piece_runs = [&](int i, std::vector<uint32_t>& runs, std::vector<uint32_t>& beg) {
        runs.clear();
        beg.assign(1, 0);
        for (uint32_t r = 0; r < R; r++) {
            const uint32_t a = cut(r, i), e = cut(r, i + 1);
            if (e == a) continue;  // no frame of run r in this piece: its slot keeps its state
            runs.push_back(r);
            beg.push_back(beg.back() + (e - a));
        }
    };
    // piece i's PCM (in the staging slot it was given) -> the caller's frames, dropped frames left as
    // they are.  The slots go to the non-empty pieces in turn (a time slice of runs shorter than P
    // frames can be empty: ADVICE r5 -- slot i % 2 by piece index lost a piece's PCM behind an empty
    // piece), and a slot is drained right before it is reused and at the end.
    std::vector<uint32_t> out_runs, out_beg;
    int slot_owner[kStageSlots];
    std::fill(slot_owner, slot_owner + kStageSlots, -1);
    int next_slot = 0;
    auto copy_out = [&](int slot) -> int {
        const int i = slot_owner[slot];
        if (i < 0) return JAAD_OK;
        slot_owner[slot] = -1;
        HIPCHK(hipEventSynchronize(ctx->ev_out[i]));
        piece_runs(i, out_runs, out_beg);
        const char* src = static_cast<const char*>(ctx->stage_out[slot].p);
        const size_t nr = out_runs.size();
        io.run([&](int t) {
            for (size_t k = nr * t / W; k < nr * (t + 1) / W; k++) {
                const uint32_t a = cut(out_runs[k], i), n = out_beg[k + 1] - out_beg[k];
                const char* sp = src + (size_t)out_beg[k] * fbytes;
                char* dp = static_cast<char*>(pcm_out) + (size_t)a * fbytes;
                if (!b->frame_status) {
                    std::memcpy(dp, sp, (size_t)n * fbytes);
                    continue;
                }
                for (uint32_t j = 0; j < n; j++)
                    if (kept(a + j)) std::memcpy(dp + (size_t)j * fbytes, sp + (size_t)j * fbytes, fbytes);
            }
        });
        return JAAD_OK;
    };
    // piece i: the runs' slices gathered into staging slot i % 2 by the workers, checked on the way
    // (side info; |q| as q_ok_copy copies it), then one H2D copy (ev_in[i])
    std::vector<uint32_t> st_runs, st_beg;
    auto stage_piece = [&](int i) -> int {
        const size_t nfi = NF[i + 1] - NF[i];
        const Layout L = layout(nfi);
        if (i >= kStageSlots) HIPCHK(hipEventSynchronize(ctx->ev_in[i - kStageSlots]));
        char* st = static_cast<char*>(ctx->stage_in[i % kStageSlots].p);
        piece_runs(i, st_runs, st_beg);
        const size_t nr = st_runs.size();
        if (!nfi) return hipEventRecord(ctx->ev_in[i], ctx->h2d) == hipSuccess ? JAAD_OK : JAAD_ERR_HIP;
        io.run([&](int t) {
            for (size_t k = nr * t / W; k < nr * (t + 1) / W; k++) {
                const size_t a = cut(st_runs[k], i), n = st_beg[k + 1] - st_beg[k], o = st_beg[k];
                const size_t c0 = a * nch, nc = n * nch, oc = o * nch;
                if (!side_info_ok(ctx, b, c0, c0 + nc)) bad = true;
                int16_t* qd = dma_q ? nullptr : reinterpret_cast<int16_t*>(st + L.q) + oc * 1024;
                if (!q_ok_copy(b->q + c0 * 1024, qd, nc * 1024)) {  // (stopped at the bad block)
                    if (!b->frame_status || !q_ok_kept(ctx, b, c0, c0 + nc)) bad = true;
                    else if (qd) std::memcpy(qd, b->q + c0 * 1024, nc * 2048);  // the bad values are in dropped frames
                }
                std::memcpy(st + L.sf + oc * 128, b->sf + c0 * 128, nc * 128);
                std::memcpy(st + L.cb + oc * 128, b->cb + c0 * 128, nc * 128);
                std::memcpy(st + L.ics + oc * sizeof(jaad_ics_info), b->ics + c0, nc * sizeof(jaad_ics_info));
                if (b->ms_used) std::memcpy(st + L.ms + o * 8 * mw, b->ms_used + a * mw, n * 8 * mw);
                if (b->tns) std::memcpy(st + L.tns + oc * sizeof(jaad_tns), b->tns + c0, nc * sizeof(jaad_tns));
            }
        });
        if (bad) return JAAD_ERR_BITSTREAM;
        if (dma_q) {  // q straight from the caller's registered memory (one range), the side info from staging
            const size_t f0 = b->frame_begin[(*run0)[i]];
            HIPCHK(hipMemcpyAsync(base + SB[i] + L.q, b->q + f0 * nch * 1024, nfi * nch * 2048, hipMemcpyHostToDevice, ctx->h2d));
            HIPCHK(hipMemcpyAsync(base + SB[i] + L.sf, st + L.sf, L.bytes - L.sf, hipMemcpyHostToDevice, ctx->h2d));
        } else {
            HIPCHK(hipMemcpyAsync(base + SB[i], st, L.bytes, hipMemcpyHostToDevice, ctx->h2d));
        }
        HIPCHK(hipEventRecord(ctx->ev_in[i], ctx->h2d));
        return JAAD_OK;
    };
    static const bool trace = std::getenv("JAAD_TRACE_HOST") != nullptr;  // per-piece host timings (tuning aid)
    using clk = std::chrono::steady_clock;
    auto ms = [](clk::time_point a, clk::time_point e) { return std::chrono::duration<double, std::milli>(e - a).count(); };
    const auto t_call = clk::now();
    int rc = stage_piece(0);
    if (rc) return rc;
    int queued = 0;
    for (int i = 0; i < P; i++) {
        const auto t0 = clk::now();
        const size_t nfi = NF[i + 1] - NF[i];
        if (!nfi) {  // (runs shorter than P frames: no frame falls in this slice)
            HIPCHK(hipEventRecord(ctx->ev_out[i], ctx->d2h));
            if (i + 1 < P && (rc = stage_piece(i + 1))) return rc;
            queued = i + 1;
            continue;
        }
        const Layout L = layout(nfi);
        const char* blk = base + SB[i];
        piece_runs(i, prun, pbeg);
        pslot.resize(prun.size());
        for (size_t k = 0; k < prun.size(); k++) pslot[k] = b->stream_slot[prun[k]];
        if (b->sbr || b->frame_status) {  // host-side per-frame arrays of the piece
            if (b->sbr) psbr.resize(nfi * sw);
            if (b->frame_status) pstat.resize(nfi);
            const size_t nr = prun.size();
            io.run([&](int t) {
                for (size_t k = nr * t / W; k < nr * (t + 1) / W; k++) {
                    const size_t a = cut(prun[k], i), n = pbeg[k + 1] - pbeg[k];
                    if (b->sbr) std::memcpy(&psbr[pbeg[k] * sw], b->sbr + a * sw, n * sw * sizeof(jaad_sbr_frame));
                    if (b->frame_status) std::memcpy(&pstat[pbeg[k]], b->frame_status + a, n);
                }
            });
        }
        jaad_batch pb = *b;  // the piece as a batch of its own
        pb.n_frames = (uint32_t)nfi;
        pb.n_runs = (uint32_t)prun.size();
        pb.stream_slot = pslot.data();
        pb.frame_begin = pbeg.data();
        pb.q = reinterpret_cast<const int16_t*>(blk + L.q);
        pb.sf = reinterpret_cast<const uint8_t*>(blk + L.sf);
        pb.cb = reinterpret_cast<const uint8_t*>(blk + L.cb);
        pb.ics = reinterpret_cast<const jaad_ics_info*>(blk + L.ics);
        pb.ms_used = b->ms_used ? reinterpret_cast<const uint64_t*>(blk + L.ms) : nullptr;
        pb.tns = b->tns ? reinterpret_cast<const jaad_tns*>(blk + L.tns) : nullptr;
        pb.sbr = b->sbr ? psbr.data() : nullptr;
        pb.frame_status = b->frame_status ? pstat.data() : nullptr;
        if (nce) {  // the piece's terms: each run's slice of frames, renumbered (terms are sorted by frame)
            pterms.clear();
            auto at = [&](uint32_t f) {
                return std::lower_bound(b->cce_terms, b->cce_terms + b->n_cce_terms, f,
                                        [](const jaad_cce_term& T, uint32_t v) { return T.frame < v; });
            };
            for (size_t k = 0; k < prun.size(); k++) {
                const uint32_t a = cut(prun[k], i), e = cut(prun[k], i + 1);
                for (const jaad_cce_term* t = at(a); t < b->cce_terms + b->n_cce_terms && t->frame < e; t++) {
                    pterms.push_back(*t);
                    pterms.back().frame = pbeg[k] + (t->frame - a);
                }
            }
            pb.n_cce_terms = (uint32_t)pterms.size();
            pb.cce_terms = pterms.data();
            pb.cce_q = reinterpret_cast<const int16_t*>(base + o_cq);
            pb.cce_sf = reinterpret_cast<const uint8_t*>(base + o_csf);
            pb.cce_cb = reinterpret_cast<const uint8_t*>(base + o_ccb);
            pb.cce_ics = reinterpret_cast<const jaad_ics_info*>(base + o_cics);
        }
        // piece i's launch first (its SBR records go to the H2D stream now, ahead of piece i+1's
        // inputs), then piece i+1's gather and copy while piece i's kernels run
        HIPCHK(hipStreamWaitEvent(s, ctx->ev_in[i], 0));
        char* dp = dpcm + NF[i] * fbytes;
        if ((rc = launch(ctx, &pb, dp, flags, s))) return rc;
        HIPCHK(hipEventRecord(ctx->ev_k[i], s));
        const auto t1 = clk::now();
        if (i + 1 < P && (rc = stage_piece(i + 1))) return rc;
        const auto t2 = clk::now();
        HIPCHK(hipStreamWaitEvent(ctx->d2h, ctx->ev_k[i], 0));
        if (dma_out && run0) {  // the piece's frames straight into the caller's registered memory
            HIPCHK(hipMemcpyAsync(static_cast<char*>(pcm_out) + (size_t)b->frame_begin[(*run0)[i]] * fbytes, dp, nfi * fbytes,
                                  hipMemcpyDeviceToHost, ctx->d2h));
        } else if (dma_out) {  // the piece's R rows straight into the caller's registered memory
            const size_t w = (size_t)(cut(0, i + 1) - cut(0, i)) * fbytes;
            HIPCHK(hipMemcpy2DAsync(static_cast<char*>(pcm_out) + (size_t)cut(0, i) * fbytes, (size_t)L0 * fbytes, dp, w, w,
                                    prun.size(), hipMemcpyDeviceToHost, ctx->d2h));
        } else {
            const int slot = next_slot;
            next_slot = (next_slot + 1) % kStageSlots;
            if ((rc = copy_out(slot))) return rc;  // drains the slot's previous piece
            slot_owner[slot] = i;
            HIPCHK(hipMemcpyAsync(ctx->stage_out[slot].p, dp, nfi * fbytes, hipMemcpyDeviceToHost, ctx->d2h));
        }
        HIPCHK(hipEventRecord(ctx->ev_out[i], ctx->d2h));
        queued = i + 1;
        if (trace)
            std::fprintf(stderr, "jaad pieces: piece %d/%d (%zu frames) at %.3f ms: launch %.3f, stage next %.3f, out %.3f ms\n", i,
                         P, nfi, ms(t_call, t0), ms(t0, t1), ms(t1, t2), ms(t2, clk::now()));
    }
    if (!dma_out)
        for (int k = 0; k < kStageSlots; k++)  // the last pieces, oldest first
            if ((rc = copy_out((next_slot + k) % kStageSlots))) return rc;
    (void)queued;
    HIPCHK(hipStreamSynchronize(ctx->d2h));
    HIPCHK(hipStreamSynchronize(s));
    if (trace) std::fprintf(stderr, "jaad pieces: call %.3f ms (q %s, PCM %s)\n", ms(t_call, clk::now()), dma_q ? "dma" : "staged",
                            dma_out ? "dma" : "staged");
    return JAAD_OK;
}

static int decode_batch_pieces_launch(jaad_ctx* ctx, const jaad_batch* b, void* pcm_out, uint32_t flags, int P,
                                      const std::vector<uint32_t>* run0)
{
    std::vector<StateSnap> snaps;
    bool saved = false;
    ctx->rec_stream = ctx->h2d;
    for (jaad_ctx* c : ctx->children) c->rec_stream = ctx->h2d;
    const int rc = decode_batch_pieces_launch_impl(ctx, b, pcm_out, flags, P, run0, snaps, saved);
    ctx->rec_stream = nullptr;
    for (jaad_ctx* c : ctx->children) c->rec_stream = nullptr;
    if (rc) {
        for (hipStream_t st : {ctx->h2d, ctx->d2h, ctx->stream})
            if (st) (void)hipStreamSynchronize(st);
        (void)hipGetLastError();
        if (saved) {  // every slot (of every element context) back to the state it had when the call started
            auto al = [](size_t x) { return (x + 255) & ~(size_t)255; };
            const char* bk = static_cast<const char*>(ctx->d_backup.p);
            for (StateSnap& S : snaps) {
                const char* o = bk + S.off;
                S.c->parity = S.parity;
                if (S.lc_b) (void)hipMemcpy(S.c->d_state[S.parity], o, S.lc_b, hipMemcpyDeviceToDevice);
                if (S.sbr_b) (void)hipMemcpy(S.c->d_sbr_state, o + al(S.lc_b), S.sbr_b, hipMemcpyDeviceToDevice);
                if (S.ps_b) (void)hipMemcpy(S.c->d_ps_state, o + al(S.lc_b) + al(S.sbr_b), S.ps_b, hipMemcpyDeviceToDevice);
                S.c->sbr_slots.swap(S.host);
            }
            (void)hipDeviceSynchronize();
        }
    }
    return rc;
}

// ---- dropped frames (jaad_batch.frame_status) ----
// A dropped frame is left out of the call's plan (keep_map): the kernels walk each run's kept
// frames as consecutive ones, so a run cut by a dropped frame continues from the state its
// previous frame left -- what the reference's next decodeFrame sees after it swallowed the
// EOSException (A/Decoder.java:89-101) -- and the dropped frame's PCM slot is not written.

// the number of dropped frames (0: none, or no status array); JAAD_ERR_INVALID_ARG (< 0) for a
// status value that is not a JAAD_FRAME_*
static int dropped_frames(const jaad_batch* b)
{
    if (!b->frame_status) return 0;
    int n = 0;
    for (uint32_t f = 0; f < b->n_frames; f++) {
        if (b->frame_status[f] > JAAD_FRAME_EOS) return JAAD_ERR_INVALID_ARG;
        n += b->frame_status[f] != JAAD_FRAME_DECODE;
    }
    return n;
}

static int decode_batch_whole(jaad_ctx* ctx, const jaad_batch* b, void* pcm_out, uint32_t flags);

// any EIGHT_SHORT frame among the batch's channel-frames (the host entry's own scan for the
// mixed-window kernel, KernelArgs::short_pair); multichannel elements decode per element and keep
// the per-channel short path
static void set_short_hint(jaad_ctx* ctx, const jaad_batch* b)
{
    bool any = false;
    if (ctx->n_elem == 1 && ctx->nch == 2 && b->ics)
        for (size_t i = 0, n = (size_t)b->n_frames * ctx->nch; i < n && !any; i++)
            any = b->ics[i].window_sequence == JAAD_EIGHT_SHORT_SEQUENCE;
    ctx->hint_short = any;
}

int jaad_decode_batch(jaad_ctx* ctx, const jaad_batch* b, void* pcm_out, size_t pcm_bytes, uint32_t flags)
{
    flags &= ~(uint32_t)JAAD_HINT_SHORT_WINDOWS;  // (a device-entry hint: the host entry scans)
    int rc = check_batch(ctx, b, pcm_bytes, flags);
    if (rc) return rc;
    set_short_hint(ctx, b);
    if (!pcm_out && b->n_frames) return JAAD_ERR_INVALID_ARG;
    const int dropped = dropped_frames(b);
    if (dropped < 0) return dropped;
    jaad_batch d = *b;
    if (!dropped) d.frame_status = nullptr;  // the kernels then read no frame map
    return decode_batch_whole(ctx, &d, pcm_out, flags);
}

static int decode_batch_whole(jaad_ctx* ctx, const jaad_batch* b, void* pcm_out, uint32_t flags)
{
    int rc;
    HIPCHK(hipSetDevice(ctx->device));
    if ((rc = io_setup(ctx))) return rc;
    if (b->n_frames < 2 * kMinPieceFrames ||
        !b->stream_slot || !b->frame_begin)
        return decode_batch_serial(ctx, b, pcm_out, flags);
    // the run layout is checked by plan(); pieces need it sane before cutting
    if (b->frame_begin[0] != 0 || b->frame_begin[b->n_runs] != b->n_frames) return JAAD_ERR_INVALID_ARG;
    for (uint32_t r = 0; r < b->n_runs; r++)
        if (b->frame_begin[r + 1] < b->frame_begin[r]) return JAAD_ERR_INVALID_ARG;
    if (ctx->cfg.ps) {  // time-sliced pieces through launch()
        const uint32_t P = std::min<uint32_t>(ctx->sbr_pieces ? std::min<uint32_t>(ctx->sbr_pieces, kMaxPieces) : 8u,
                                              b->n_frames / kMinPieceFrames);
        if (P < 2) return decode_batch_serial(ctx, b, pcm_out, flags);
        return decode_batch_pieces_launch(ctx, b, pcm_out, flags, (int)P, nullptr);
    }
    if (ctx->cfg.sbr || b->frame_status || ctx->n_elem > 1 || b->n_cce_terms) {  // run-aligned pieces through launch()
        const std::vector<uint32_t> run0 = cut_pieces(b);
        if (run0.size() <= 2) return decode_batch_serial(ctx, b, pcm_out, flags);
        return decode_batch_pieces_launch(ctx, b, pcm_out, flags, (int)run0.size() - 1, &run0);
    }
    const std::vector<uint32_t> run0 = cut_pieces(b);
    if (run0.size() <= 2) return decode_batch_serial(ctx, b, pcm_out, flags);
    return decode_batch_pieces(ctx, b, pcm_out, flags, run0);
}

static std::vector<jaad_ctx::PinRange>::iterator find_pin(jaad_ctx* ctx, void* p);

int jaad_host_register(jaad_ctx* ctx, void* p, size_t bytes)
{
    if (!ctx || !p || !bytes) return JAAD_ERR_INVALID_ARG;
    {  // a second registration of the same range is a no-op (one entry, one unregister)
        auto it = find_pin(ctx, p);
        if (it != ctx->pinned.end()) return it->n >= bytes ? JAAD_OK : JAAD_ERR_INVALID_ARG;
    }
    HIPCHK(hipSetDevice(ctx->device));
    // memory that is page-locked already (hipHostMalloc, another registration) is recorded as is
    hipPointerAttribute_t at{};
    if (hipPointerGetAttributes(&at, p) == hipSuccess && at.type == hipMemoryTypeHost) {
        ctx->pinned.push_back({reinterpret_cast<uintptr_t>(p), bytes, kPinForeign});
        return JAAD_OK;
    }
    (void)hipGetLastError();  // pageable memory: the query's error is expected
    HIPCHK(hipHostRegister(p, bytes, hipHostRegisterDefault));
    ctx->pinned.push_back({reinterpret_cast<uintptr_t>(p), bytes, kPinRegistered});
    return JAAD_OK;
}

static std::vector<jaad_ctx::PinRange>::iterator find_pin(jaad_ctx* ctx, void* p)
{
    return std::find_if(ctx->pinned.begin(), ctx->pinned.end(),
                        [&](const jaad_ctx::PinRange& r) { return r.p == reinterpret_cast<uintptr_t>(p); });
}

int jaad_host_unregister(jaad_ctx* ctx, void* p)
{
    if (!ctx || !p) return JAAD_ERR_INVALID_ARG;
    auto it = find_pin(ctx, p);
    if (it == ctx->pinned.end() || it->kind == kPinOwned) return JAAD_ERR_INVALID_ARG;
    HIPCHK(hipSetDevice(ctx->device));
    if (ctx->done_live) HIPCHK(hipEventSynchronize(ctx->done));
    const int kind = it->kind;
    ctx->pinned.erase(it);
    if (kind == kPinRegistered) HIPCHK(hipHostUnregister(p));
    return JAAD_OK;
}

int jaad_host_alloc(jaad_ctx* ctx, size_t bytes, void** p)
{
    if (!ctx || !bytes || !p) return JAAD_ERR_INVALID_ARG;
    *p = nullptr;
    HIPCHK(hipSetDevice(ctx->device));
    void* q = nullptr;
    if (hipHostMalloc(&q, bytes, hipHostMallocDefault) != hipSuccess || !q) {
        (void)hipGetLastError();
        return JAAD_ERR_NOMEM;
    }
    ctx->pinned.push_back({reinterpret_cast<uintptr_t>(q), bytes, kPinOwned});
    *p = q;
    return JAAD_OK;
}

int jaad_host_free(jaad_ctx* ctx, void* p)
{
    if (!ctx || !p) return JAAD_ERR_INVALID_ARG;
    auto it = find_pin(ctx, p);
    if (it == ctx->pinned.end() || it->kind != kPinOwned) return JAAD_ERR_INVALID_ARG;
    HIPCHK(hipSetDevice(ctx->device));
    if (ctx->done_live) HIPCHK(hipEventSynchronize(ctx->done));
    ctx->pinned.erase(it);
    HIPCHK(hipHostFree(p));
    return JAAD_OK;
}

int jaad_decode_batch_device(jaad_ctx* ctx, const jaad_batch* b, void* pcm_dev, size_t pcm_bytes, uint32_t flags,
                             void* hip_stream)
{
    const bool hint = (flags & JAAD_HINT_SHORT_WINDOWS) != 0;
    flags &= ~(uint32_t)JAAD_HINT_SHORT_WINDOWS;
    int rc = check_batch(ctx, b, pcm_bytes, flags);
    if (rc) return rc;
    if (ctx) ctx->hint_short = hint && ctx->n_elem == 1 && ctx->nch == 2;
    if (!pcm_dev && b->n_frames) return JAAD_ERR_INVALID_ARG;
    HIPCHK(hipSetDevice(ctx->device));
    hipStream_t s = hip_stream ? static_cast<hipStream_t>(hip_stream) : ctx->stream;
    const int dropped = dropped_frames(b);
    if (dropped < 0) return dropped;
    jaad_batch d = *b;
    if (!dropped) d.frame_status = nullptr;
    return launch(ctx, &d, pcm_dev, flags, s);
}

int jaad_wait(jaad_ctx* ctx)
{
    if (!ctx) return JAAD_ERR_INVALID_ARG;
    return sync_ctx(ctx);
}

int jaad_ctx_core_channels(const jaad_ctx* ctx) { return ctx ? ctx->nch : JAAD_ERR_INVALID_ARG; }

// per-slot state blob: core overlap [2][1024] f32 | (SBR) device SbrChState[2] | host SbrHostSlot
// | (PS) device PsState | trailer (round 6, ADVICE r5: a blob names its layout version and the
// context kind it was written by; an import checks both, so a blob of another build or of another
// kind of context is refused instead of being read as raw struct bytes)
struct StateTrailer {
    uint32_t magic, version, kind, payload;
};
constexpr uint32_t kStateMagic = 0x4441414Au;  // "JAAD"
constexpr uint32_t kStateVersion = 6;          // layout of round 6 (SbrHostSlot with blim_hw)
static size_t state_payload_bytes(const jaad_ctx* ctx)
{
    return (size_t)ctx->n_elem * 2048 * sizeof(float) + (ctx->cfg.sbr ? 2 * sizeof(SbrChState) + sizeof(SbrHostSlot) : 0) +
           (ctx->cfg.ps ? sizeof(PsState) : 0);
}
static StateTrailer state_trailer(const jaad_ctx* ctx)
{
    const uint32_t kind = (uint32_t)ctx->n_elem | (uint32_t)ctx->cfg.sbr << 8 | (uint32_t)ctx->cfg.ps << 9 |
                          (uint32_t)sbr_downsampled(ctx->cfg) << 10 | (uint32_t)ctx->cfg.ext_sf_index << 16;
    return StateTrailer{kStateMagic, kStateVersion, kind, (uint32_t)state_payload_bytes(ctx)};
}

size_t jaad_state_bytes(const jaad_ctx* ctx)
{
    if (!ctx) return 0;
    if (!ctx->children.empty()) {  // multichannel HE-AAC: the elements' blobs back to back
        size_t n = 0;
        for (const jaad_ctx* c : ctx->children) n += jaad_state_bytes(c);
        return n;
    }
    return state_payload_bytes(ctx) + sizeof(StateTrailer);
}

int jaad_state_export(jaad_ctx* ctx, uint32_t slot, void* buf, size_t bytes)
{
    if (!ctx || !buf || slot >= ctx->n_slots || bytes < jaad_state_bytes(ctx)) return JAAD_ERR_INVALID_ARG;
    int rc = sync_ctx(ctx);
    if (rc) return rc;
    char* o = static_cast<char*>(buf);
    if (!ctx->children.empty()) {
        for (jaad_ctx* c : ctx->children) {
            const size_t n = jaad_state_bytes(c);
            if ((rc = jaad_state_export(c, slot, o, n))) return rc;
            o += n;
        }
        return JAAD_OK;
    }
    for (int k = 0; k < ctx->n_elem; k++)  // one overlap record per channel element
        HIPCHK(hipMemcpy(o + (size_t)k * 2048 * sizeof(float), ctx->d_state[ctx->parity] + ((size_t)k * ctx->n_slots + slot) * 2048,
                         2048 * sizeof(float), hipMemcpyDeviceToHost));
    if (ctx->cfg.sbr) {
        char* q = o + 2048 * sizeof(float);
        HIPCHK(hipMemcpy(q, ctx->d_sbr_state + (size_t)slot * 2, 2 * sizeof(SbrChState), hipMemcpyDeviceToHost));
        std::memcpy(q + 2 * sizeof(SbrChState), &ctx->sbr_slots[slot], sizeof(SbrHostSlot));
        if (ctx->cfg.ps)
            HIPCHK(hipMemcpy(q + 2 * sizeof(SbrChState) + sizeof(SbrHostSlot), ctx->d_ps_state + slot, sizeof(PsState),
                             hipMemcpyDeviceToHost));
    }
    const StateTrailer t = state_trailer(ctx);
    std::memcpy(o + state_payload_bytes(ctx), &t, sizeof t);
    return JAAD_OK;
}

// a state blob's checks (finite overlap, a table set this context can derive from its SBR header):
// all of them run before anything is written, so a refused import leaves the slot (and, for a
// multichannel context, every element's slot) as it was
static int state_blob_check(jaad_ctx* ctx, const char* in, SbrHostSlot* hs)
{
    StateTrailer t;
    std::memcpy(&t, in + state_payload_bytes(ctx), sizeof t);
    const StateTrailer want = state_trailer(ctx);
    if (t.magic != want.magic || t.version != want.version || t.kind != want.kind || t.payload != want.payload)
        return JAAD_ERR_INVALID_ARG;
    for (int k = 0; k < ctx->n_elem; k++) {  // the overlap must be finite (the LC kernel's PCM rounding relies on it, jaad_lc.hip round_pk16)
        float ov[2048];
        std::memcpy(ov, in + (size_t)k * sizeof ov, sizeof ov);
        for (float v : ov)
            if (!std::isfinite(v)) return JAAD_ERR_INVALID_ARG;
    }
    if (ctx->cfg.sbr) {
        std::memcpy(hs, in + 2048 * sizeof(float) + 2 * sizeof(SbrChState), sizeof *hs);
        if (hs->have_hdr) {  // re-derive the table index in this context from the saved header(s)
            hs->table = ctx->sbr_host->table_index(*hs);
            if (hs->table < 0) return JAAD_ERR_INVALID_ARG;
        }
        // the PS kernels skip bands at or above the stream's band high-water mark; an imported
        // value is not trusted (a lower one would drop live all-pass state): all 64 bands, which
        // decodes identically (a band that never had input keeps zero state either way)
        hs->blim_hw = 64;
    }
    return JAAD_OK;
}

static int state_blob_apply(jaad_ctx* ctx, uint32_t slot, const char* in, const SbrHostSlot& hs)
{
    for (int k = 0; k < ctx->n_elem; k++)
        HIPCHK(hipMemcpy(ctx->d_state[ctx->parity] + ((size_t)k * ctx->n_slots + slot) * 2048, in + (size_t)k * 2048 * sizeof(float),
                         2048 * sizeof(float), hipMemcpyHostToDevice));
    if (ctx->cfg.sbr) {
        in += 2048 * sizeof(float);
        HIPCHK(hipMemcpy(ctx->d_sbr_state + (size_t)slot * 2, in, 2 * sizeof(SbrChState), hipMemcpyHostToDevice));
        if (ctx->cfg.ps)
            HIPCHK(hipMemcpy(ctx->d_ps_state + slot, in + 2 * sizeof(SbrChState) + sizeof(SbrHostSlot), sizeof(PsState),
                             hipMemcpyHostToDevice));
        ctx->sbr_slots[slot] = hs;
    }
    return JAAD_OK;
}

int jaad_state_import(jaad_ctx* ctx, uint32_t slot, const void* buf, size_t bytes)
{
    if (!ctx || !buf || slot >= ctx->n_slots || bytes < jaad_state_bytes(ctx)) return JAAD_ERR_INVALID_ARG;
    int rc = sync_ctx(ctx);
    if (rc) return rc;
    const char* in = static_cast<const char*>(buf);
    if (!ctx->children.empty()) {
        std::vector<SbrHostSlot> hs(ctx->children.size());
        const char* p = in;
        for (size_t k = 0; k < ctx->children.size(); k++) {  // every element's blob first
            jaad_ctx* c = ctx->children[k];
            if ((rc = sync_ctx(c)) || (rc = state_blob_check(c, p, &hs[k]))) return rc;
            p += jaad_state_bytes(c);
        }
        for (size_t k = 0; k < ctx->children.size(); k++) {
            jaad_ctx* c = ctx->children[k];
            if ((rc = state_blob_apply(c, slot, in, hs[k]))) return rc;
            in += jaad_state_bytes(c);
        }
        return JAAD_OK;
    }
    SbrHostSlot hs{};
    if ((rc = state_blob_check(ctx, in, &hs))) return rc;
    return state_blob_apply(ctx, slot, in, hs);
}

int jaad_state_reset(jaad_ctx* ctx, uint32_t slot)
{
    if (!ctx || slot >= ctx->n_slots) return JAAD_ERR_INVALID_ARG;
    int rc = sync_ctx(ctx);
    if (rc) return rc;
    if (!ctx->children.empty()) {
        for (jaad_ctx* c : ctx->children)
            if ((rc = jaad_state_reset(c, slot))) return rc;
        return JAAD_OK;
    }
    for (int k = 0; k < ctx->n_elem; k++)
        HIPCHK(hipMemset(ctx->d_state[ctx->parity] + ((size_t)k * ctx->n_slots + slot) * 2048, 0, 2048 * sizeof(float)));
    if (ctx->cfg.sbr) {
        HIPCHK(hipMemset(ctx->d_sbr_state + (size_t)slot * 2, 0, 2 * sizeof(SbrChState)));
        SbrHost::reset_slot(ctx->sbr_slots[slot]);
        if (ctx->cfg.ps) HIPCHK(hipMemset(ctx->d_ps_state + slot, 0, sizeof(PsState)));
    }
    return JAAD_OK;
}

}  // extern "C"
