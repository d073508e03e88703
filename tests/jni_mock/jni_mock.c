/* TEST INFRASTRUCTURE: the mock JNIEnv behind tests/test_jni_glue.py.  A "direct ByteBuffer" is
 * a jni_mock_buffer {address, capacity}; FindClass returns the class name; ThrowNew records the
 * pending exception (class and message) for the test to read. */
#include <string.h>

#include "jni.h"

typedef struct jni_mock_buffer {
    void* address;
    jlong capacity;
} jni_mock_buffer;

static char g_class[256], g_msg[1024];
static int g_pending;

static jclass find_class(JNIEnv* env, const char* name) { (void)env; return (jclass)name; }
static jint throw_new(JNIEnv* env, jclass cls, const char* msg)
{
    (void)env;
    strncpy(g_class, (const char*)cls, sizeof g_class - 1);
    strncpy(g_msg, msg, sizeof g_msg - 1);
    g_pending = 1;
    return 0;
}
static void* buf_address(JNIEnv* env, jobject b) { (void)env; return b ? ((jni_mock_buffer*)b)->address : 0; }
static jlong buf_capacity(JNIEnv* env, jobject b) { (void)env; return b ? ((jni_mock_buffer*)b)->capacity : -1; }

/* buffers made by NewDirectByteBuffer: a small pool the test reads back with jni_mock_buffer_at */
static jni_mock_buffer g_made[16];
static int g_n_made;
static jobject new_direct(JNIEnv* env, void* address, jlong capacity)
{
    (void)env;
    if (g_n_made >= 16) return 0;
    g_made[g_n_made].address = address;
    g_made[g_n_made].capacity = capacity;
    return &g_made[g_n_made++];
}

static const struct JNINativeInterface_ g_table = {find_class, throw_new, buf_address, buf_capacity, new_direct};
static JNIEnv g_env = &g_table;

JNIEXPORT JNIEnv* jni_mock_env(void) { return &g_env; }
/* the pending exception: 1 and its class / message, or 0; clears it */
JNIEXPORT int jni_mock_take_exception(char* cls, int cls_len, char* msg, int msg_len)
{
    const int p = g_pending;
    if (p) {
        strncpy(cls, g_class, cls_len - 1);
        cls[cls_len - 1] = 0;
        strncpy(msg, g_msg, msg_len - 1);
        msg[msg_len - 1] = 0;
    }
    g_pending = 0;
    g_class[0] = g_msg[0] = 0;
    return p;
}
