/* tests/jni_harness/jni.h — TEST INFRASTRUCTURE: the subset of the JNI API that integration/jvm/native/
 * sparkts_arima_jni.c uses, so the shim compiles and its exports can be driven without a JVM (no JDK in this image).
 * The real build (integration/jvm/native/Makefile) uses the JDK's jni.h; this struct is NOT the JDK's function-table
 * layout -- it only serves the harness's fake environment (jni_env.c). */
#ifndef SPARKTS_TEST_JNI_H
#define SPARKTS_TEST_JNI_H
#include <stddef.h>  /* the JDK jni.h pulls in stdio.h/stdarg.h, hence NULL */
#include <stdint.h>

#define JNIEXPORT __attribute__((visibility("default")))
#define JNICALL
typedef int32_t jint;
typedef int64_t jlong;
typedef uint8_t jboolean;
typedef void *jobject;
typedef jobject jstring;

struct JNINativeInterface_;
typedef const struct JNINativeInterface_ *JNIEnv;
struct JNINativeInterface_ {
    void *(*GetDirectBufferAddress)(JNIEnv *env, jobject buf);
    jstring (*NewStringUTF)(JNIEnv *env, const char *utf);
    const char *(*GetStringUTFChars)(JNIEnv *env, jstring str, jboolean *is_copy);
    void (*ReleaseStringUTFChars)(JNIEnv *env, jstring str, const char *chars);
};
#endif
