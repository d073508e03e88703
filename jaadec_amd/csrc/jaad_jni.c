/* JNI glue for the reference's Java side: net.sourceforge.jaad.aac.gpu.GpuDSP.
 *
 * Compiled only where a JDK is installed (build.py looks for $JAVA_HOME/include/jni.h; this
 * image has none, so here it is documentation that build.py skips).  Every buffer crosses as a
 * direct java.nio.ByteBuffer in native byte order: no copies, no pinning, no JNI arrays.
 * A nonzero jaad_status becomes net.sourceforge.jaad.aac.AACException (A/AACException.java),
 * the exception Decoder.decodeFrame's callers already handle (A/Decoder.java:86-101).
 */
#include <jni.h>
#include <stdint.h>
#include <stdio.h>
#include <string.h>

#include "jaad_gpu.h"

static void throw_aac(JNIEnv* env, jaad_ctx* ctx, int status) {
    char msg[512];
    const char* detail = ctx ? jaad_last_error(ctx) : "";
    snprintf(msg, sizeof msg, "%s%s%s", jaad_strerror(status), detail && *detail ? ": " : "", detail ? detail : "");
    jclass cls = (*env)->FindClass(env, "net/sourceforge/jaad/aac/AACException");
    if (cls) (*env)->ThrowNew(env, cls, msg);
}

static void* addr(JNIEnv* env, jobject bb, jlong need) {
    if (!bb) return NULL;
    if ((*env)->GetDirectBufferCapacity(env, bb) < need) return NULL;
    return (*env)->GetDirectBufferAddress(env, bb);
}

/* static native long nativeCreate(int sfIndex, int channelConfig, int tnsMode, int sbr, int ps,
 *     int precision, int nSlots, int device); sfIndex is the core (AAC) rate, the SBR rate is twice
 *     it; precision = JAAD_PRECISION_EXACT (0) or JAAD_PRECISION_LSB1 (1) */
JNIEXPORT jlong JNICALL Java_net_sourceforge_jaad_aac_gpu_GpuDSP_nativeCreate(JNIEnv* env, jclass cls, jint sf_index,
                                                                            jint channel_config, jint tns_mode,
                                                                            jint sbr, jint ps, jint precision,
                                                                            jint n_slots, jint device) {
    (void)cls;
    jaad_stream_cfg cfg;
    memset(&cfg, 0, sizeof cfg);
    cfg.abi_version = JAAD_ABI_VERSION;
    cfg.profile = 2;
    cfg.sf_index = (uint8_t)sf_index;
    cfg.channel_config = (uint8_t)channel_config;
    cfg.tns_mode = (uint8_t)tns_mode;
    cfg.sbr = (uint8_t)(sbr || ps);
    cfg.ps = (uint8_t)ps;
    cfg.ext_sf_index = (uint8_t)(cfg.sbr ? sf_index - 3 : 0);
    cfg.precision = (uint8_t)precision;  /* jaad_ctx_create rejects values other than 0 / 1 */
    jaad_ctx* ctx = NULL;
    int rc = jaad_ctx_create(&cfg, (uint32_t)n_slots, device, &ctx);
    if (rc) {
        throw_aac(env, NULL, rc);
        return 0;
    }
    return (jlong)(intptr_t)ctx;
}

JNIEXPORT void JNICALL Java_net_sourceforge_jaad_aac_gpu_GpuDSP_nativeDestroy(JNIEnv* env, jclass cls, jlong h) {
    (void)env;
    (void)cls;
    jaad_ctx_destroy((jaad_ctx*)(intptr_t)h);
}

/* ms_used pairs per frame: one per CPE of the configuration (core channels 2: 1; 3, 4: 1; 5, 6: 2;
 * 8: 3; mono: none) */
static int cpe_count(int nch) { return nch == 1 ? 0 : nch <= 4 ? 1 : nch <= 6 ? 2 : 3; }

/* the batch of a decode call; with n_terms > 0 the coupling records and terms too */
static void decode_common(JNIEnv* env, jaad_ctx* ctx, jint n_frames, jint n_runs, jint nch, jobject stream_slot,
                          jobject frame_begin, jobject q, jobject sf, jobject cb, jobject ics, jobject ms_used,
                          jobject tns, jobject sbr, jobject pcm, jint flags, jint n_cce, jint n_terms, jobject cce_q,
                          jobject cce_sf, jobject cce_cb, jobject cce_ics, jobject cce_terms, jobject frame_status) {
    if (!ctx || n_frames < 0 || n_runs < 0 || n_cce < 0 || n_terms < 0 || nch != jaad_ctx_core_channels(ctx)) {
        throw_aac(env, ctx, JAAD_ERR_INVALID_ARG);
        return;
    }
    const jlong ncf = (jlong)n_frames * nch;
    jaad_batch b;
    memset(&b, 0, sizeof b);
    b.n_frames = (uint32_t)n_frames;
    b.n_runs = (uint32_t)n_runs;
    b.stream_slot = (const uint32_t*)addr(env, stream_slot, 4LL * n_runs);
    b.frame_begin = (const uint32_t*)addr(env, frame_begin, 4LL * (n_runs + 1));
    b.q = (const int16_t*)addr(env, q, 2048LL * ncf);
    b.sf = (const uint8_t*)addr(env, sf, 128LL * ncf);
    b.cb = (const uint8_t*)addr(env, cb, 128LL * ncf);
    b.ics = (const jaad_ics_info*)addr(env, ics, (jlong)sizeof(jaad_ics_info) * ncf);
    b.ms_used = (const uint64_t*)addr(env, ms_used, 16LL * n_frames * (cpe_count(nch) ? cpe_count(nch) : 1));
    b.tns = (const jaad_tns*)addr(env, tns, (jlong)sizeof(jaad_tns) * ncf);
    b.sbr = (const jaad_sbr_frame*)addr(env, sbr, (jlong)sizeof(jaad_sbr_frame) * n_frames);
    if (n_terms) {
        b.n_cce = (uint32_t)n_cce;
        b.n_cce_terms = (uint32_t)n_terms;
        b.cce_q = (const int16_t*)addr(env, cce_q, 2048LL * n_cce);
        b.cce_sf = (const uint8_t*)addr(env, cce_sf, 128LL * n_cce);
        b.cce_cb = (const uint8_t*)addr(env, cce_cb, 128LL * n_cce);
        b.cce_ics = (const jaad_ics_info*)addr(env, cce_ics, (jlong)sizeof(jaad_ics_info) * n_cce);
        b.cce_terms = (const jaad_cce_term*)addr(env, cce_terms, (jlong)sizeof(jaad_cce_term) * n_terms);
    }
    b.frame_status = (const uint8_t*)addr(env, frame_status, (jlong)n_frames);
    jlong pcm_cap = pcm ? (*env)->GetDirectBufferCapacity(env, pcm) : -1;
    void* out = pcm ? (*env)->GetDirectBufferAddress(env, pcm) : NULL;
    if (!b.stream_slot || !b.frame_begin || !b.q || !b.sf || !b.cb || !b.ics || !out || pcm_cap < 0 ||
        (ms_used && !b.ms_used) || (tns && !b.tns) || (sbr && !b.sbr) || (frame_status && !b.frame_status) ||
        (n_terms && (!b.cce_q || !b.cce_sf || !b.cce_cb || !b.cce_ics || !b.cce_terms))) {
        throw_aac(env, ctx, JAAD_ERR_INVALID_ARG);
        return;
    }
    int rc = jaad_decode_batch(ctx, &b, out, (size_t)pcm_cap, (uint32_t)flags);
    if (rc) throw_aac(env, ctx, rc);
}

/* static native void nativeDecode(long h, int nFrames, int nRuns, int nch, ByteBuffer streamSlot,
 *     ByteBuffer frameBegin, ByteBuffer q, ByteBuffer sf, ByteBuffer cb, ByteBuffer ics,
 *     ByteBuffer msUsed, ByteBuffer tns, ByteBuffer sbr, ByteBuffer pcm, int flags,
 *     ByteBuffer frameStatus);
 * nch: channels per frame (1 SCE core, 2 CPE core, 3..8 multichannel); must equal the context's
 * (jaad_ctx_core_channels), since every buffer capacity below is checked against it.
 * sbr: one jaad_sbr_frame (1968 B, sizeof(jaad_sbr_frame)) per frame for SBR/PS streams, else null.
 * frameStatus: one byte per frame (JAAD_FRAME_EOS = 1 for a frame whose parse threw EOSException:
 * dropped, its PCM slot left as it is) or null when every frame decodes. */
JNIEXPORT void JNICALL Java_net_sourceforge_jaad_aac_gpu_GpuDSP_nativeDecode(
    JNIEnv* env, jclass cls, jlong h, jint n_frames, jint n_runs, jint nch, jobject stream_slot, jobject frame_begin,
    jobject q, jobject sf, jobject cb, jobject ics, jobject ms_used, jobject tns, jobject sbr, jobject pcm, jint flags,
    jobject frame_status) {
    (void)cls;
    decode_common(env, (jaad_ctx*)(intptr_t)h, n_frames, n_runs, nch, stream_slot, frame_begin, q, sf, cb, ics, ms_used,
                  tns, sbr, pcm, flags, 0, 0, NULL, NULL, NULL, NULL, NULL, frame_status);
}

/* static native void nativeDecodeCoupled(long h, int nFrames, int nRuns, int nch, ByteBuffer streamSlot,
 *     ByteBuffer frameBegin, ByteBuffer q, ByteBuffer sf, ByteBuffer cb, ByteBuffer ics,
 *     ByteBuffer msUsed, ByteBuffer tns, ByteBuffer sbr, ByteBuffer pcm, int flags, int nCce,
 *     int nTerms, ByteBuffer cceQ, ByteBuffer cceSf, ByteBuffer cceCb, ByteBuffer cceIcs,
 *     ByteBuffer cceTerms, ByteBuffer frameStatus);
 * a batch with coupling channel elements: nCce CCE ICStream records and nTerms jaad_cce_term
 * (488 B) in the reference's order (jaad_gpu.h); sbr and frameStatus as nativeDecode's (null sbr
 * for AAC-LC; coupling is applied to the core spectra before the SBR/PS stage either way) */
JNIEXPORT void JNICALL Java_net_sourceforge_jaad_aac_gpu_GpuDSP_nativeDecodeCoupled(
    JNIEnv* env, jclass cls, jlong h, jint n_frames, jint n_runs, jint nch, jobject stream_slot, jobject frame_begin,
    jobject q, jobject sf, jobject cb, jobject ics, jobject ms_used, jobject tns, jobject sbr, jobject pcm, jint flags,
    jint n_cce, jint n_terms, jobject cce_q, jobject cce_sf, jobject cce_cb, jobject cce_ics, jobject cce_terms,
    jobject frame_status) {
    (void)cls;
    decode_common(env, (jaad_ctx*)(intptr_t)h, n_frames, n_runs, nch, stream_slot, frame_begin, q, sf, cb, ics, ms_used,
                  tns, sbr, pcm, flags, n_cce, n_terms, cce_q, cce_sf, cce_cb, cce_ics, cce_terms, frame_status);
}

/* static native int nativeStateBytes(long h): size of one slot's state blob (jaad_state_bytes).
 * static native void nativeStateExport(long h, int slot, ByteBuffer buf) /
 * nativeStateImport(long h, int slot, ByteBuffer buf): a stream's DSP state (IMDCT overlap,
 * window shape, SBR/PS filterbank and envelope state) out to / back from a direct buffer of at
 * least nativeStateBytes bytes -- seek/resume of one stream (jaad_state_export / import). */
JNIEXPORT jint JNICALL Java_net_sourceforge_jaad_aac_gpu_GpuDSP_nativeStateBytes(JNIEnv* env, jclass cls, jlong h) {
    (void)cls;
    jaad_ctx* ctx = (jaad_ctx*)(intptr_t)h;
    if (!ctx) {
        throw_aac(env, ctx, JAAD_ERR_INVALID_ARG);
        return 0;
    }
    return (jint)jaad_state_bytes(ctx);
}

static void state_io(JNIEnv* env, jlong h, jint slot, jobject buf, int do_export) {
    jaad_ctx* ctx = (jaad_ctx*)(intptr_t)h;
    const jlong cap = buf ? (*env)->GetDirectBufferCapacity(env, buf) : -1;
    void* p = buf ? (*env)->GetDirectBufferAddress(env, buf) : NULL;
    if (!ctx || !p || cap < 0 || slot < 0) {
        throw_aac(env, ctx, JAAD_ERR_INVALID_ARG);
        return;
    }
    const size_t n = jaad_state_bytes(ctx);
    if ((size_t)cap < n) {
        throw_aac(env, ctx, JAAD_ERR_INVALID_ARG);
        return;
    }
    const int rc = do_export ? jaad_state_export(ctx, (uint32_t)slot, p, n) : jaad_state_import(ctx, (uint32_t)slot, p, n);
    if (rc) throw_aac(env, ctx, rc);
}

JNIEXPORT void JNICALL Java_net_sourceforge_jaad_aac_gpu_GpuDSP_nativeStateExport(JNIEnv* env, jclass cls, jlong h,
                                                                                jint slot, jobject buf) {
    (void)cls;
    state_io(env, h, slot, buf, 1);
}

JNIEXPORT void JNICALL Java_net_sourceforge_jaad_aac_gpu_GpuDSP_nativeStateImport(JNIEnv* env, jclass cls, jlong h,
                                                                                jint slot, jobject buf) {
    (void)cls;
    state_io(env, h, slot, buf, 0);
}

JNIEXPORT void JNICALL Java_net_sourceforge_jaad_aac_gpu_GpuDSP_nativeReset(JNIEnv* env, jclass cls, jlong h,
                                                                          jint slot) {
    (void)cls;
    jaad_ctx* ctx = (jaad_ctx*)(intptr_t)h;
    int rc = jaad_state_reset(ctx, (uint32_t)slot);
    if (rc) throw_aac(env, ctx, rc);
}

/* static native void nativeRegister(long h, ByteBuffer buf) / nativeUnregister(long h, ByteBuffer buf):
 * page-lock a direct buffer the stream reuses call after call (jaad_host_register), so
 * nativeDecode copies it by DMA without staging; unregister before the buffer is released. */
JNIEXPORT void JNICALL Java_net_sourceforge_jaad_aac_gpu_GpuDSP_nativeRegister(JNIEnv* env, jclass cls, jlong h,
                                                                             jobject buf) {
    (void)cls;
    jaad_ctx* ctx = (jaad_ctx*)(intptr_t)h;
    const jlong cap = buf ? (*env)->GetDirectBufferCapacity(env, buf) : -1;
    void* p = buf ? (*env)->GetDirectBufferAddress(env, buf) : NULL;
    const int rc = (!ctx || !p || cap <= 0) ? JAAD_ERR_INVALID_ARG : jaad_host_register(ctx, p, (size_t)cap);
    if (rc) throw_aac(env, ctx, rc);
}

JNIEXPORT void JNICALL Java_net_sourceforge_jaad_aac_gpu_GpuDSP_nativeUnregister(JNIEnv* env, jclass cls, jlong h,
                                                                               jobject buf) {
    (void)cls;
    jaad_ctx* ctx = (jaad_ctx*)(intptr_t)h;
    void* p = buf ? (*env)->GetDirectBufferAddress(env, buf) : NULL;
    const int rc = (!ctx || !p) ? JAAD_ERR_INVALID_ARG : jaad_host_unregister(ctx, p);
    if (rc) throw_aac(env, ctx, rc);
}

/* static native ByteBuffer nativeAllocDirect(long h, long bytes) / nativeFreeDirect(long h, ByteBuffer buf):
 * a direct buffer over page-locked memory the context owns (jaad_host_alloc): a stream that
 * keeps its q/side-info/PCM arrays in such buffers gets DMA without staging and without
 * registering pageable memory.  Free it (nativeFreeDirect) before dropping the buffer;
 * nativeDestroy frees what is left. */
JNIEXPORT jobject JNICALL Java_net_sourceforge_jaad_aac_gpu_GpuDSP_nativeAllocDirect(JNIEnv* env, jclass cls, jlong h,
                                                                                   jlong bytes) {
    (void)cls;
    jaad_ctx* ctx = (jaad_ctx*)(intptr_t)h;
    void* p = NULL;
    const int rc = (!ctx || bytes <= 0) ? JAAD_ERR_INVALID_ARG : jaad_host_alloc(ctx, (size_t)bytes, &p);
    if (rc) {
        throw_aac(env, ctx, rc);
        return NULL;
    }
    jobject buf = (*env)->NewDirectByteBuffer(env, p, bytes);
    if (!buf) (void)jaad_host_free(ctx, p);  /* the JVM has an OutOfMemoryError pending */
    return buf;
}

JNIEXPORT void JNICALL Java_net_sourceforge_jaad_aac_gpu_GpuDSP_nativeFreeDirect(JNIEnv* env, jclass cls, jlong h,
                                                                               jobject buf) {
    (void)cls;
    jaad_ctx* ctx = (jaad_ctx*)(intptr_t)h;
    void* p = buf ? (*env)->GetDirectBufferAddress(env, buf) : NULL;
    const int rc = (!ctx || !p) ? JAAD_ERR_INVALID_ARG : jaad_host_free(ctx, p);
    if (rc) throw_aac(env, ctx, rc);
}
