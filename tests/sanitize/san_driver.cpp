// san_driver.cpp — TEST INFRASTRUCTURE (sanitizers on host code). Built with
// -fsanitize=address,undefined together with the CPU restatement (oracle/arima_oracle.c) and the kernel's optimizer
// state machine on the CPU (tests/sim/cglane_sim.cpp, which includes spark-timeseries_amd/csrc/cg_lane.hpp), so
// every array, union member and slot index those two touch is checked while they fit a spread of orders, lengths
// and edge inputs (T = 0..16, NaN, constant, failing and MaxEval fits). It also checks that the state machine
// reproduces the restatement's fits bit for bit on the same series (status, n_eval, n_grad, coefficients, LL), so
// a sanitizer-clean run is also a parity run. Exit status 0 = clean and identical; any sanitizer report aborts.
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

extern "C" {
int orc_fit(const double *ts, int T, int p, int d, int q, int I, int method, const double *user_init, int smear,
            double *coef_out, double *ll_out, int *counters);
int orc_hannan_rissanen(const double *y, int n, int p, int q, int I, double *params);
void orc_differences_of_order_d(const double *ts, int T, int d, double *out);
void orc_inverse_differences_of_order_d(const double *in, int L, int d, double *out);
void orc_gradient_css_arma(const double *y, int n, int p, int q, int I, const double *coef, int smear,
                           double *grad);
double orc_loglik_css_arma(const double *y, int n, int p, int q, int I, const double *coef);
void orc_forecast(const double *ts, int T, int p, int d, int q, int I, const double *coef, int nFuture,
                  double *out);
void orc_add_time_dependent_effects(const double *ts, int n, int p, int d, int q, int I, const double *coef,
                                    double *out);
int orc_lag_matrix(const double *x, int n, int maxLag, int includeOriginal, double *out_colmajor);
int sim_fit_batch(const double *y, int64_t N, int ld, int n, int p, int q, int I, int smear, const double *init,
                  int ns, int nc, double *coef, double *ll, int32_t *status, int32_t *counts);
int sim_nan_iter_evals(int dir_finite);
int sim_k_nan_iter_evals();
}

namespace {

uint64_t g_state = 0x9E3779B97F4A7C15ull;
double unif() {                                      // splitmix64 -> [0, 1)
    uint64_t z = (g_state += 0x9E3779B97F4A7C15ull);
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    z ^= z >> 31;
    return (double)(z >> 11) * (1.0 / 9007199254740992.0);
}
double normal() {
    double u = unif(), v = unif();
    if (u < 1e-300) u = 1e-300;
    return std::sqrt(-2.0 * std::log(u)) * std::cos(6.283185307179586 * v);
}

bool same(double a, double b) {
    uint64_t x, y;
    std::memcpy(&x, &a, 8);
    std::memcpy(&y, &b, 8);
    return x == y || (std::isnan(a) && std::isnan(b));
}

int failures = 0, compared = 0, converged = 0, failed_fits = 0;

// one series: the restatement's fit, and the state machine's fit from the same HR init under two speculation
// policies (the kernel's NS = 2 / NC = 4, and none), compared field by field
void check_series(const std::vector<double> &ts, int p, int d, int q, int I, int smear, const char *what) {
    const int T = (int)ts.size(), k = I + p + q;
    double coef[16], ll;
    int cnt[3];
    const int st = orc_fit(ts.empty() ? nullptr : ts.data(), T, p, d, q, I, 0, nullptr, smear, coef, &ll, cnt);
    if (T < d || k == 0 || (p > 0 && q == 0)) return;        // no CG fit to compare (shape error / AR shortcut)
    const int n = T - d;
    std::vector<double> diff((size_t)T + 1), y((size_t)n + 1);
    orc_differences_of_order_d(ts.data(), T, d, diff.data());
    for (int i = 0; i < n; ++i) y[i] = diff[d + i];
    double init[16];
    if (orc_hannan_rissanen(y.data(), n, p, q, I, init) != 0) return;
    for (int pol = 0; pol < 2; ++pol) {
        double c[16], l;
        int32_t s, counts[14];
        sim_fit_batch(y.data(), 1, n, n, p, q, I, smear, init, pol ? 2 : 0, pol ? 4 : 0, c, &l, &s, counts);
        bool ok = s == st && counts[0] == cnt[0] && counts[1] == cnt[1];
        ++compared;
        if (pol == 0) (st == 0 ? converged : failed_fits)++;
        for (int j = 0; j < k && ok; ++j) ok = same(c[j], coef[j]);
        if (ok && st == 0) ok = same(l, ll);
        if (!ok) {
            std::printf("MISMATCH %s (%d,%d,%d)+%d T=%d smear=%d policy=%d: status %d/%d evals %d/%d grads %d/%d\n",
                        what, p, d, q, I, T, smear, pol, (int)s, st, counts[0], cnt[0], counts[1], cnt[1]);
            ++failures;
        }
    }
}

std::vector<double> arima_series(int T, int p, int d, int q, int I) {
    const int k = I + p + q;
    double c[16];
    for (int j = 0; j < k; ++j) c[j] = (j < I) ? 2.0 : 0.35 / (1 + j);
    const int n = T - d > 0 ? T - d : 0;
    std::vector<double> noise((size_t)n + 1), out((size_t)n + 1);
    for (int i = 0; i < n; ++i) noise[i] = normal();
    orc_add_time_dependent_effects(noise.data(), n, p, d, q, I, c, out.data());
    std::vector<double> ts((size_t)T, 0.0);
    for (int i = 0; i < n; ++i) ts[d + i] = out[i];
    return ts;
}

}  // namespace

int main() {
    // orders x lengths (short series hit every shape error of ARIMA.scala:216-242 and commons' OLS checks)
    const int orders[][4] = {{1, 0, 1, 1}, {2, 1, 2, 1}, {0, 1, 1, 1}, {3, 0, 0, 1}, {0, 0, 0, 1}, {0, 0, 0, 0},
                             {5, 1, 5, 1}, {2, 2, 4, 0}, {4, 1, 3, 0}, {1, 2, 0, 0}, {0, 0, 5, 1}, {5, 0, 2, 1}};
    const int lengths[] = {0, 1, 2, 3, 4, 5, 6, 7, 8, 9, 10, 11, 12, 13, 14, 15, 16, 40, 300};
    for (const auto &o : orders)
        for (int T : lengths)
            for (int smear = 0; smear <= 1; ++smear) {
                std::vector<double> ts = arima_series(T, o[0], o[1], o[2], o[3]);
                check_series(ts, o[0], o[1], o[2], o[3], smear, "synthetic");
            }
    // edge inputs: NaN inside, all-constant, huge scale
    for (const auto &o : orders) {
        std::vector<double> ts = arima_series(120, o[0], o[1], o[2], o[3]);
        std::vector<double> nan_ts = ts;
        nan_ts[60] = NAN;
        check_series(nan_ts, o[0], o[1], o[2], o[3], 1, "nan");
        std::vector<double> flat(120, 3.25);
        check_series(flat, o[0], o[1], o[2], o[3], 1, "constant");
        for (double &v : ts) v *= 1e150;
        check_series(ts, o[0], o[1], o[2], o[3], 1, "huge");
    }
    // css-bobyqa (oracle/bobyqa_oracle.c): every array of Powell's routines under the sanitizers, over the orders,
    // short and edge series (its results are checked against the device by tests/test_gpu_bobyqa.py)
    for (const auto &o : orders)
        for (int T : {0, 3, 9, 16, 40, 300}) {
            std::vector<double> ts = arima_series(T, o[0], o[1], o[2], o[3]);
            double coef[16], ll;
            int cnt[3];
            orc_fit(ts.empty() ? nullptr : ts.data(), T, o[0], o[1], o[2], o[3], 1, nullptr, 1, coef, &ll, cnt);
            std::vector<double> flat(T > 0 ? T : 1, 3.25), nan_ts = ts;
            orc_fit(T ? flat.data() : nullptr, T, o[0], o[1], o[2], o[3], 1, nullptr, 1, coef, &ll, cnt);
            if (T > 20) {
                nan_ts[T / 2] = NAN;
                orc_fit(nan_ts.data(), T, o[0], o[1], o[2], o[3], 1, nullptr, 1, coef, &ll, cnt);
            }
        }
    // building blocks the fit does not reach on its own
    for (const auto &o : orders) {
        const int p = o[0], d = o[1], q = o[2], I = o[3], k = I + p + q;
        std::vector<double> ts = arima_series(64, p, d, q, I);
        double c[16], g[16];
        for (int j = 0; j < k; ++j) c[j] = 0.1 * (j + 1);
        std::vector<double> y((size_t)ts.size() + 1);
        orc_differences_of_order_d(ts.data(), (int)ts.size(), d, y.data());
        for (int smear = 0; smear <= 1; ++smear) orc_gradient_css_arma(y.data() + d, 64 - d, p, q, I, c, smear, g);
        (void)orc_loglik_css_arma(y.data() + d, 64 - d, p, q, I, c);
        std::vector<double> fc(64 + 17);
        orc_forecast(ts.data(), 64, p, d, q, I, c, 17, fc.data());
        std::vector<double> inv(64);
        orc_inverse_differences_of_order_d(y.data(), 64, d, inv.data());
        std::vector<double> lag(64 * 8);
        orc_lag_matrix(ts.data(), 10, 3, 1, lag.data());
        orc_lag_matrix(ts.data(), 10, 3, 0, lag.data());
    }
    // the NaN fast-forward constant, stepped without the shortcut
    for (int f = 0; f <= 1; ++f)
        if (sim_nan_iter_evals(f) != sim_k_nan_iter_evals()) {
            std::printf("MISMATCH nan_iter_evals(%d)\n", f);
            ++failures;
        }
    std::printf("san_driver: %d fits compared (%d converged, %d failed), %d mismatches\n", compared, converged,
                failed_fits, failures);
    return (failures || compared < 100 || failed_fits == 0) ? 1 : 0;
}
