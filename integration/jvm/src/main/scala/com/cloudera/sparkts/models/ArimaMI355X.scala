/*
 * ArimaMI355X.scala — the reference-side binding of the MI355X engine (spark-ts 0.4.0-SNAPSHOT, Scala 2.11).
 *
 * A maintainer drops this file into spark-ts (src/main/scala/com/cloudera/sparkts/models/) together with
 * libsparkts_arima.so and libsparkts_arima_jni.so (integration/jvm/native). It cannot be compiled in the build
 * container of this repository (no JDK / Scala / jars); the C ABI it calls is tested there through ctypes.
 *
 *   ArimaMI355X.fitModel(p, d, q, ts, ...)     drop-in for ARIMA.fitModel (ARIMA.scala:79-116), one series
 *   ArimaMI355X.mapSeriesFit(rdd, p, d, q)     drop-in for tsrdd.mapSeries(v => Vectors.dense(
 *                                              ARIMA.fitModel(p, d, q, v).coefficients)) (TimeSeriesRDD.scala:249-251,
 *                                              JavaTimeSeriesRDD.scala:124-133), batched per partition
 *   ArimaMI355X.forecastMany / orderSearchMany batched ARIMAModel.forecast (ARIMA.scala:696-764) and the
 *                                              min-approxAIC order grid (ARIMA.scala:280-375, 826-830)
 *   ArimaMI355X.autoFit / autoFitMany          drop-in for ARIMA.autoFit (ARIMA.scala:280-375): KPSS choice of d,
 *                                              stepwise walk with the css-bobyqa retry, batched per partition
 *   method = "css-bobyqa"                      fitWithCSSBOBYQA (ARIMA.scala:130-160) on the device
 */
package com.cloudera.sparkts.models

import java.nio.{ByteBuffer, ByteOrder, DoubleBuffer, IntBuffer}

import org.apache.commons.math3.exception.{MathIllegalArgumentException, NoDataException,
  NumberIsTooLargeException, TooManyEvaluationsException, TooManyIterationsException}
import org.apache.commons.math3.exception.util.LocalizedFormats
import org.apache.commons.math3.linear.SingularMatrixException
import org.apache.spark.mllib.linalg.{Vector, Vectors}
import org.apache.spark.rdd.RDD

/** JNI entry points (integration/jvm/native/sparkts_arima_jni.c -> include/sparkts_arima.h). */
object ArimaMI355XNative {
  System.loadLibrary("sparkts_arima_jni")
  @native def create(device: Int): Long
  @native def destroy(handle: Long): Int
  @native def lastError(handle: Long): String
  @native def setOption(handle: Long, name: String, value: Long): Int
  @native def fitBatch(handle: Long, series: DoubleBuffer, n: Long, t: Int, p: Int, d: Int, q: Int,
                       intercept: Boolean, method: Int, userInit: DoubleBuffer, coef: DoubleBuffer,
                       ll: DoubleBuffer, status: IntBuffer, nEval: IntBuffer, nGrad: IntBuffer,
                       flags: ByteBuffer): Int
  @native def forecastBatch(handle: Long, series: DoubleBuffer, n: Long, t: Int, p: Int, d: Int, q: Int,
                            intercept: Boolean, coef: DoubleBuffer, nFuture: Int, out: DoubleBuffer): Int
  @native def orderSearch(handle: Long, series: DoubleBuffer, n: Long, t: Int, maxP: Int, maxD: Int, maxQ: Int,
                          interceptMode: Int, method: Int, order: IntBuffer, coef: DoubleBuffer,
                          aic: DoubleBuffer): Int
  @native def autoFit(handle: Long, series: DoubleBuffer, n: Long, t: Int, maxP: Int, maxD: Int, maxQ: Int,
                      order: IntBuffer, coef: DoubleBuffer, aic: DoubleBuffer, status: IntBuffer,
                      nFits: IntBuffer): Int
}

/** Per-series status codes of include/sparkts_arima.h, mapped back to the exception the reference throws. */
object ArimaStatus {
  val OK = 0; val MAX_EVAL = 1; val BRACKET_MAX_EVAL = 2; val MAX_ITER = 3; val SINGULAR = 4
  val NOT_ENOUGH_DATA = 5; val NO_DATA = 6; val BAD_INTERVAL = 7; val ZERO_PARAMS = 8
  val UNSUPPORTED_METHOD = 9; val SERIES_TOO_SHORT = 10
  val NOT_STATIONARY = 11; val NO_MODEL = 12; val TOO_FEW_PARAMS = 14     // 13, 15 retired (RESCUE restated)

  def toException(status: Int): Throwable = status match {
    case MAX_EVAL => new TooManyEvaluationsException(10000)                    // MaxEval(10000), ARIMA.scala:196
    case BRACKET_MAX_EVAL => new TooManyEvaluationsException(500)              // BracketFinder's own cap
    case MAX_ITER => new TooManyIterationsException(10000)                     // MaxIter(10000), ARIMA.scala:195
    case SINGULAR => new SingularMatrixException()                             // OLS QR, ARIMA.scala:237-240
    case NOT_ENOUGH_DATA => new MathIllegalArgumentException(LocalizedFormats.NOT_ENOUGH_DATA_FOR_NUMBER_OF_PREDICTORS, 0: Integer, 0: Integer)
    case NO_DATA => new NoDataException()
    case BAD_INTERVAL => new NumberIsTooLargeException(0.0, 0.0, false)        // SearchInterval in LineSearch
    case ZERO_PARAMS => new ArithmeticException("/ by zero")
    case UNSUPPORTED_METHOD => new UnsupportedOperationException()             // ARIMA.scala:108
    case SERIES_TOO_SHORT => new IndexOutOfBoundsException()
    case NOT_STATIONARY => new Exception("stationarity not achieved with differencing order <= maxD")  // :295
    case NO_MODEL => new NullPointerException()                                // curBestModel == null, :302
    case TOO_FEW_PARAMS => new org.apache.commons.math3.exception.NumberIsTooSmallException(1: Integer, 2: Integer, true)
    case other => new IllegalStateException(s"unknown ARIMA status $other")
  }
}

object ArimaMI355X {
  /** One engine handle per executor JVM; the handle serialises calls, so task threads may share it. */
  private lazy val handle: Long = {
    val dev = sys.env.getOrElse("SPARKTS_DEVICE", "0").toInt      // one executor per GPU
    val h = ArimaMI355XNative.create(dev)
    require(h != 0L, s"arima_create(device = $dev) failed")
    h
  }

  private def methodCode(method: String): Int = method match {
    case "css-cgd" => 0
    case "css-bobyqa" => 1                                        // fitWithCSSBOBYQA, ARIMA.scala:130-160
    case _ => 99                                                  // -> UNSUPPORTED_METHOD, as ARIMA.scala:108
  }

  private def doubles(len: Long): DoubleBuffer = {
    require(len * 8 <= Int.MaxValue, "batch too large for one direct buffer: split the partition")
    ByteBuffer.allocateDirect((len * 8).toInt).order(ByteOrder.nativeOrder).asDoubleBuffer
  }

  private def ints(len: Long): IntBuffer =
    ByteBuffer.allocateDirect((len * 4).toInt).order(ByteOrder.nativeOrder).asIntBuffer

  private def check(rc: Int, what: String): Unit =
    if (rc != 0) throw new IllegalStateException(s"$what failed ($rc): ${ArimaMI355XNative.lastError(handle)}")

  /** Result of one batched fit: coefficients in the reference layout [c?, phi_1..phi_p, theta_1..theta_q]
    * (ARIMA.scala:74-77, 406), CSS log-likelihood, per-series status and the reference's evaluation counters. */
  case class FitResult(coefficients: Array[Array[Double]], cssLogLikelihood: Array[Double], status: Array[Int],
                       nEval: Array[Int], nGrad: Array[Int])

  /** Drop-in for ARIMA.fitModel (ARIMA.scala:79-116): a batch of one, same exceptions. */
  def fitModel(p: Int, d: Int, q: Int, ts: Vector, includeIntercept: Boolean = true,
               method: String = "css-cgd", userInitParams: Array[Double] = null): ARIMAModel = {
    val r = fitMany(p, d, q, Array(ts.toArray), includeIntercept, method, userInitParams)
    if (r.status(0) != ArimaStatus.OK) throw ArimaStatus.toException(r.status(0))
    new ARIMAModel(p, d, q, r.coefficients(0), includeIntercept)
  }

  /** One ABI call (arima_fit_batch) for a bucket of equal-length series, packed series-major N x T. */
  def fitMany(p: Int, d: Int, q: Int, values: Array[Array[Double]], includeIntercept: Boolean = true,
              method: String = "css-cgd", userInitParams: Array[Double] = null): FitResult = {
    val n = values.length
    val t = if (n == 0) 0 else values(0).length
    require(values.forall(_.length == t), "one call takes series of equal length (bucket by length)")
    val k = p + q + (if (includeIntercept) 1 else 0)
    val series = doubles(n.toLong * t)
    values.foreach(v => series.put(v))
    series.flip()
    val ui = if (userInitParams == null) null else {
      require(userInitParams.length == k, s"userInitParams must have $k entries")
      val b = doubles(n.toLong * k)
      (0 until n).foreach(_ => b.put(userInitParams))
      b.flip()
      b
    }
    val coef = doubles(math.max(n.toLong * k, 1L))
    val ll = doubles(math.max(n, 1))
    val status = ints(math.max(n, 1))
    val nEval = ints(math.max(n, 1))
    val nGrad = ints(math.max(n, 1))
    check(ArimaMI355XNative.fitBatch(handle, series, n, t, p, d, q, includeIntercept, methodCode(method), ui,
      coef, ll, status, nEval, nGrad, null), "arima_fit_batch")
    FitResult(Array.tabulate(n)(i => Array.tabulate(k)(j => coef.get(i * k + j))), Array.tabulate(n)(ll.get),
      Array.tabulate(n)(status.get), Array.tabulate(n)(nEval.get), Array.tabulate(n)(nGrad.get))
  }

  /** Drop-in for `tsrdd.mapSeries(v => Vectors.dense(ARIMA.fitModel(p, d, q, v).coefficients))`: per partition,
    * bucket the records by length, one ABI call per bucket; keys and record order are preserved. A series whose
    * fit fails gets NaN coefficients (the reference closure would have thrown; wrap it in Try to compare). */
  def mapSeriesFit[K](rdd: RDD[(K, Vector)], p: Int, d: Int, q: Int, includeIntercept: Boolean = true,
                      method: String = "css-cgd"): RDD[(K, Vector)] = rdd.mapPartitions { it =>
    val recs = it.toArray
    val out = new Array[(K, Vector)](recs.length)
    recs.indices.groupBy(i => recs(i)._2.size).foreach { case (_, idx) =>
      val r = fitMany(p, d, q, idx.map(i => recs(i)._2.toArray).toArray, includeIntercept, method, null)
      idx.zipWithIndex.foreach { case (i, j) => out(i) = (recs(i)._1, Vectors.dense(r.coefficients(j))) }
    }
    out.iterator
  }

  /** Batched ARIMAModel.forecast (ARIMA.scala:696-764): N x (T + nFuture). */
  def forecastMany(model: ARIMAModel, values: Array[Array[Double]], nFuture: Int): Array[Array[Double]] = {
    val n = values.length
    val t = if (n == 0) 0 else values(0).length
    val k = model.coefficients.length
    val series = doubles(n.toLong * t)
    values.foreach(v => series.put(v))
    series.flip()
    val coef = doubles(math.max(n.toLong * k, 1L))
    (0 until n).foreach(_ => coef.put(model.coefficients))
    coef.flip()
    val out = doubles(math.max(n.toLong * (t + nFuture), 1L))
    check(ArimaMI355XNative.forecastBatch(handle, series, n, t, model.p, model.d, model.q, model.hasIntercept,
      coef, nFuture, out), "arima_forecast_batch")
    Array.tabulate(n)(i => Array.tabulate(t + nFuture)(j => out.get(i * (t + nFuture) + j)))
  }

  /** Drop-in for ARIMA.autoFit (ARIMA.scala:280-304): one series, the reference's exceptions. maxP <= 8 (its
    * css-bobyqa retries have at most 11 parameters). */
  def autoFit(ts: Vector, maxP: Int = 5, maxD: Int = 2, maxQ: Int = 5): ARIMAModel = {
    val (order, coef, _, status) = autoFitMany(Array(ts.toArray), maxP, maxD, maxQ)
    val st = status(0)
    if (st != ArimaStatus.OK) throw ArimaStatus.toException(st)
    val Array(p, d, q, c) = order(0)
    new ARIMAModel(p, d, q, coef(0).take(p + q + c), c == 1)
  }

  /** Batched ARIMA.autoFit: (p, d, q, intercept), coefficients (11, zero-padded), approxAIC and status per series. */
  def autoFitMany(values: Array[Array[Double]], maxP: Int = 5, maxD: Int = 2, maxQ: Int = 5)
      : (Array[Array[Int]], Array[Array[Double]], Array[Double], Array[Int]) = {
    val n = values.length
    val t = if (n == 0) 0 else values(0).length
    val series = doubles(n.toLong * t)
    values.foreach(v => series.put(v))
    series.flip()
    val order = ints(math.max(4L * n, 1L))
    val coef = doubles(math.max(11L * n, 1L))
    val aic = doubles(math.max(n, 1))
    val status = ints(math.max(n, 1))
    val nFits = ints(math.max(n, 1))
    check(ArimaMI355XNative.autoFit(handle, series, n, t, maxP, maxD, maxQ, order, coef, aic, status, nFits),
      "arima_autofit_batch")
    (Array.tabulate(n)(i => Array.tabulate(4)(j => order.get(4 * i + j))),
      Array.tabulate(n)(i => Array.tabulate(11)(j => coef.get(11 * i + j))), Array.tabulate(n)(aic.get),
      Array.tabulate(n)(status.get))
  }

  /** The min-approxAIC (ARIMA.scala:826-830) model per series over d <= maxD, p <= maxP, q <= maxQ and the
    * intercept modes, among fits that returned normally and are stationary and invertible (ARIMA.scala:342).
    * Returns (p, d, q, intercept) per series (-1s when nothing qualified), coefficients and AIC. */
  def orderSearchMany(values: Array[Array[Double]], maxP: Int = 5, maxD: Int = 2, maxQ: Int = 5,
                      interceptMode: Int = 2): (Array[Array[Int]], Array[Array[Double]], Array[Double]) = {
    val n = values.length
    val t = if (n == 0) 0 else values(0).length
    val series = doubles(n.toLong * t)
    values.foreach(v => series.put(v))
    series.flip()
    val order = ints(math.max(4L * n, 1L))
    val coef = doubles(math.max(11L * n, 1L))
    val aic = doubles(math.max(n, 1))
    check(ArimaMI355XNative.orderSearch(handle, series, n, t, maxP, maxD, maxQ, interceptMode, 0, order, coef, aic),
      "arima_order_search_batch")
    (Array.tabulate(n)(i => Array.tabulate(4)(j => order.get(4 * i + j))),
      Array.tabulate(n)(i => Array.tabulate(11)(j => coef.get(11 * i + j))), Array.tabulate(n)(aic.get))
  }
}
