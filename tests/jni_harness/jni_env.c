/* tests/jni_harness/jni_env.c — TEST INFRASTRUCTURE: a fake JNIEnv for driving the JNI shim from Python (ctypes):
 * a "direct buffer" jobject is the buffer's address itself and a jstring is a C string. */
#include <string.h>

#include "jni.h"

static void *buf_addr(JNIEnv *env, jobject b) { (void)env; return b; }
static jstring new_str(JNIEnv *env, const char *s) { (void)env; return (jstring)s; }
static const char *str_chars(JNIEnv *env, jstring s, jboolean *c) { (void)env; if (c) *c = 0; return (const char *)s; }
static void str_release(JNIEnv *env, jstring s, const char *c) { (void)env; (void)s; (void)c; }

static const struct JNINativeInterface_ g_fns = {buf_addr, new_str, str_chars, str_release};
static JNIEnv g_env = &g_fns;

JNIEXPORT JNIEnv *fake_jni_env(void) { return &g_env; }
