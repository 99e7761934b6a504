/*
 * sparkts_arima_jni.c — JNI shim between the Scala facade (ArimaMI355X.scala, this directory's ../src) and the
 * C ABI of the MI355X engine (include/sparkts_arima.h). It only forwards: direct NIO buffers are passed through as
 * plain pointers (no copies across JNI), return codes are returned unchanged. Build (needs a JDK):
 *     make -C integration/jvm/native JAVA_HOME=/path/to/jdk
 * The JVM method owner is the Scala object `ArimaMI355XNative`, whose JVM class is `ArimaMI355XNative$`
 * (hence `_00024` in the symbol names).
 *
 * Replaces, per call: ARIMA.fitModel over a bucket of equal-length series (ARIMA.scala:79-116),
 * ARIMAModel.forecast (ARIMA.scala:696-764) and the order-search grid (ARIMA.scala:280-375, 826-830).
 */
#include <jni.h>
#include <stdint.h>

#include "sparkts_arima.h"

#define BUF(env, b) ((b) ? (*(env))->GetDirectBufferAddress((env), (b)) : NULL)
#define JNI_FN(name) Java_com_cloudera_sparkts_models_ArimaMI355XNative_00024_##name

JNIEXPORT jlong JNICALL JNI_FN(create)(JNIEnv *env, jobject self, jint device) {
    (void)env; (void)self;
    arima_handle *h = NULL;
    return arima_create(device, &h) == ARIMA_OK ? (jlong)(intptr_t)h : 0;
}

JNIEXPORT jint JNICALL JNI_FN(destroy)(JNIEnv *env, jobject self, jlong h) {
    (void)env; (void)self;
    return arima_destroy((arima_handle *)(intptr_t)h);
}

JNIEXPORT jstring JNICALL JNI_FN(lastError)(JNIEnv *env, jobject self, jlong h) {
    (void)self;
    return (*env)->NewStringUTF(env, arima_last_error((const arima_handle *)(intptr_t)h));
}

JNIEXPORT jint JNICALL JNI_FN(setOption)(JNIEnv *env, jobject self, jlong h, jstring name, jlong value) {
    (void)self;
    const char *s = (*env)->GetStringUTFChars(env, name, NULL);
    const int rc = arima_set_option((arima_handle *)(intptr_t)h, s, value);
    (*env)->ReleaseStringUTFChars(env, name, s);
    return rc;
}

/* arima_fit_batch: series N x T (DoubleBuffer), userInit N x k or null, outputs coef N x k, ll N, status N,
 * nEval / nGrad / flags N or null */
JNIEXPORT jint JNICALL JNI_FN(fitBatch)(JNIEnv *env, jobject self, jlong h, jobject series, jlong n, jint t,
                                        jint p, jint d, jint q, jboolean intercept, jint method, jobject userInit,
                                        jobject coef, jobject ll, jobject status, jobject nEval, jobject nGrad,
                                        jobject flags) {
    (void)self;
    return arima_fit_batch((arima_handle *)(intptr_t)h, (const double *)BUF(env, series), n, t, p, d, q,
                           intercept ? 1 : 0, method, (const double *)BUF(env, userInit), (double *)BUF(env, coef),
                           (double *)BUF(env, ll), (int32_t *)BUF(env, status), (int32_t *)BUF(env, nEval),
                           (int32_t *)BUF(env, nGrad), (uint8_t *)BUF(env, flags));
}

/* arima_forecast_batch: series N x T, coef N x k, out N x (T + nFuture) */
JNIEXPORT jint JNICALL JNI_FN(forecastBatch)(JNIEnv *env, jobject self, jlong h, jobject series, jlong n, jint t,
                                             jint p, jint d, jint q, jboolean intercept, jobject coef,
                                             jint nFuture, jobject out) {
    (void)self;
    return arima_forecast_batch((arima_handle *)(intptr_t)h, (const double *)BUF(env, series), n, t, p, d, q,
                                intercept ? 1 : 0, (const double *)BUF(env, coef), nFuture,
                                (double *)BUF(env, out));
}

/* arima_order_search_batch: series N x T, order N x 4, coef N x 11, aic N */
JNIEXPORT jint JNICALL JNI_FN(orderSearch)(JNIEnv *env, jobject self, jlong h, jobject series, jlong n, jint t,
                                           jint maxP, jint maxD, jint maxQ, jint interceptMode, jint method,
                                           jobject order, jobject coef, jobject aic) {
    (void)self;
    return arima_order_search_batch((arima_handle *)(intptr_t)h, (const double *)BUF(env, series), n, t, maxP,
                                    maxD, maxQ, interceptMode, method, (int32_t *)BUF(env, order),
                                    (double *)BUF(env, coef), (double *)BUF(env, aic));
}

/* arima_autofit_batch (ARIMA.autoFit, ARIMA.scala:280-375): series N x T, order N x 4, coef N x 11, aic / status /
 * n_fits N */
JNIEXPORT jint JNICALL JNI_FN(autoFit)(JNIEnv *env, jobject self, jlong h, jobject series, jlong n, jint t, jint maxP,
                                       jint maxD, jint maxQ, jobject order, jobject coef, jobject aic, jobject status,
                                       jobject nFits) {
    (void)self;
    return arima_autofit_batch((arima_handle *)(intptr_t)h, (const double *)BUF(env, series), n, t, maxP, maxD,
                               maxQ, (int32_t *)BUF(env, order), (double *)BUF(env, coef), (double *)BUF(env, aic),
                               (int32_t *)BUF(env, status), (int32_t *)BUF(env, nFits));
}
