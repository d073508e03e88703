/* TEST INFRASTRUCTURE: a minimal stand-in for a JDK's <jni.h>, enough to compile
 * jaadec_amd/csrc/jaad_jni.c without a JDK and drive it from tests/test_jni_glue.py.
 * Only the types and the JNIEnv functions the glue calls exist; the function table is this
 * mock's own (not the JVM's layout), filled in by jni_mock.c. */
#ifndef JAAD_JNI_MOCK_H
#define JAAD_JNI_MOCK_H
#include <stdint.h>

typedef int32_t jint;
typedef int64_t jlong;
typedef void* jobject;
typedef jobject jclass;

struct JNINativeInterface_;
typedef const struct JNINativeInterface_* JNIEnv;
struct JNINativeInterface_ {
    jclass (*FindClass)(JNIEnv* env, const char* name);
    jint (*ThrowNew)(JNIEnv* env, jclass cls, const char* msg);
    void* (*GetDirectBufferAddress)(JNIEnv* env, jobject buf);
    jlong (*GetDirectBufferCapacity)(JNIEnv* env, jobject buf);
    jobject (*NewDirectByteBuffer)(JNIEnv* env, void* address, jlong capacity);
};

#define JNIEXPORT __attribute__((visibility("default")))
#define JNICALL
#endif
