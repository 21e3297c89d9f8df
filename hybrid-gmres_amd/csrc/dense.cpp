// Small dense host linear algebra for the projected problems (k <= maxit, O(k^3) flops):
// the reference calls MATLAB's `\` (mldivide) and `svd` on (k+1) x k / k x k matrices
// (hybrid_ba_gmres_rtp.m:29, hybrid_ab_gmres_rtp.m:32, *_bounds.m:35-36,
// gcv_function.m:38,42, hybrid_lsmr_solver.m:44).  These stay on the host (SURVEY.md
// §8(a) A6/A8): they are latency-only and far below one kernel launch.
#include <algorithm>
#include <cmath>
#include <limits>
#include <vector>

#include "internal.h"

namespace hgm {
namespace dense {

#define AT(M, ld, i, j) (M)[(size_t)(j) * (ld) + (i)]

static bool cholesky_solve(int n, const double* Min, const double* b, double* x) {
    // LAPACK dpotrf 'U' order: R^T R = M, R upper
    std::vector<double> R(Min, Min + (size_t)n * n);
    for (int j = 0; j < n; ++j) {
        double s = AT(R.data(), n, j, j);
        for (int k = 0; k < j; ++k) s -= AT(R.data(), n, k, j) * AT(R.data(), n, k, j);
        if (!(s > 0)) return false;
        const double rjj = std::sqrt(s);
        AT(R.data(), n, j, j) = rjj;
        for (int i = j + 1; i < n; ++i) {
            double t = AT(R.data(), n, j, i);
            for (int k = 0; k < j; ++k) t -= AT(R.data(), n, k, j) * AT(R.data(), n, k, i);
            AT(R.data(), n, j, i) = t / rjj;
        }
    }
    std::vector<double> z(b, b + n);
    for (int i = 0; i < n; ++i) {           // R^T z = b
        double t = z[i];
        for (int k = 0; k < i; ++k) t -= AT(R.data(), n, k, i) * z[k];
        z[i] = t / AT(R.data(), n, i, i);
    }
    for (int i = n - 1; i >= 0; --i) {      // R x = z
        double t = z[i];
        for (int k = i + 1; k < n; ++k) t -= AT(R.data(), n, i, k) * x[k];
        x[i] = t / AT(R.data(), n, i, i);
    }
    return true;
}

static void lu_solve(int n, const double* Min, const double* b, double* x) {
    std::vector<double> M(Min, Min + (size_t)n * n);
    std::vector<double> r(b, b + n);
    for (int k = 0; k < n; ++k) {
        int p = k;
        double best = std::fabs(AT(M.data(), n, k, k));
        for (int i = k + 1; i < n; ++i)
            if (std::fabs(AT(M.data(), n, i, k)) > best) { best = std::fabs(AT(M.data(), n, i, k)); p = i; }
        if (p != k) {
            for (int j = 0; j < n; ++j) std::swap(AT(M.data(), n, k, j), AT(M.data(), n, p, j));
            std::swap(r[k], r[p]);
        }
        const double piv = AT(M.data(), n, k, k);
        for (int i = k + 1; i < n; ++i) {
            const double l = AT(M.data(), n, i, k) / piv;
            AT(M.data(), n, i, k) = l;
            for (int j = k + 1; j < n; ++j) AT(M.data(), n, i, j) -= l * AT(M.data(), n, k, j);
            r[i] -= l * r[k];
        }
    }
    for (int i = n - 1; i >= 0; --i) {
        double t = r[i];
        for (int j = i + 1; j < n; ++j) t -= AT(M.data(), n, i, j) * x[j];
        x[i] = t / AT(M.data(), n, i, i);
    }
}

void mldivide_square(int n, const double* M, const double* b, double* x) {
    if (n <= 0) return;
    bool sym = true, posdiag = true;
    for (int j = 0; j < n && sym; ++j) {
        if (!(AT(M, n, j, j) > 0)) posdiag = false;
        for (int i = j + 1; i < n; ++i)
            if (AT(M, n, i, j) != AT(M, n, j, i)) { sym = false; break; }
    }
    if (sym && posdiag && cholesky_solve(n, M, b, x)) return;
    lu_solve(n, M, b, x);
}

void qr_ls(int m, int n, const double* Min, const double* b, double* x) {
    // Householder QR with column pivoting (xGEQP3 semantics, as MATLAB's rectangular `\`).
    std::vector<double> M(Min, Min + (size_t)m * n);
    std::vector<double> r(b, b + m);
    std::vector<int> piv(n);
    std::vector<double> cn(n);
    for (int j = 0; j < n; ++j) {
        piv[j] = j;
        double s = 0;
        for (int i = 0; i < m; ++i) s += AT(M.data(), m, i, j) * AT(M.data(), m, i, j);
        cn[j] = s;
    }
    const int kmax = std::min(m, n);
    for (int k = 0; k < kmax; ++k) {
        int p = k;
        for (int j = k + 1; j < n; ++j) if (cn[j] > cn[p]) p = j;
        if (p != k) {
            for (int i = 0; i < m; ++i) std::swap(AT(M.data(), m, i, k), AT(M.data(), m, i, p));
            std::swap(piv[k], piv[p]);
            std::swap(cn[k], cn[p]);
        }
        double alpha = 0;
        for (int i = k; i < m; ++i) alpha += AT(M.data(), m, i, k) * AT(M.data(), m, i, k);
        alpha = std::sqrt(alpha);
        if (alpha == 0) continue;
        const double x0 = AT(M.data(), m, k, k);
        const double beta = x0 > 0 ? -alpha : alpha;     // R(k,k) = beta
        // v = x - beta e1, normalised so v(0) = 1
        const double v0 = x0 - beta;
        std::vector<double> v(m - k);
        v[0] = 1.0;
        for (int i = k + 1; i < m; ++i) v[i - k] = AT(M.data(), m, i, k) / v0;
        const double tau = (beta - x0) / beta;
        AT(M.data(), m, k, k) = beta;
        for (int i = k + 1; i < m; ++i) AT(M.data(), m, i, k) = 0;
        for (int j = k + 1; j < n; ++j) {
            double s = 0;
            for (int i = k; i < m; ++i) s += v[i - k] * AT(M.data(), m, i, j);
            s *= tau;
            for (int i = k; i < m; ++i) AT(M.data(), m, i, j) -= s * v[i - k];
        }
        {
            double s = 0;
            for (int i = k; i < m; ++i) s += v[i - k] * r[i];
            s *= tau;
            for (int i = k; i < m; ++i) r[i] -= s * v[i - k];
        }
        for (int j = k + 1; j < n; ++j) {       // downdate remaining column norms
            double s = 0;
            for (int i = k + 1; i < m; ++i) s += AT(M.data(), m, i, j) * AT(M.data(), m, i, j);
            cn[j] = s;
        }
    }
    std::vector<double> z(n, 0.0);
    for (int i = kmax - 1; i >= 0; --i) {
        double t = r[i];
        for (int j = i + 1; j < kmax; ++j) t -= AT(M.data(), m, i, j) * z[j];
        const double d = AT(M.data(), m, i, i);
        z[i] = d != 0 ? t / d : 0.0;
    }
    for (int j = 0; j < n; ++j) x[piv[j]] = z[j];
}

void svd_values(int n, const double* Min, double* s) {
    // one-sided Jacobi on the columns
    std::vector<double> U(Min, Min + (size_t)n * n);
    const double eps = std::numeric_limits<double>::epsilon();
    for (int sweep = 0; sweep < 60; ++sweep) {
        double off = 0;
        for (int p = 0; p < n - 1; ++p)
            for (int q = p + 1; q < n; ++q) {
                double a = 0, b = 0, g = 0;
                for (int i = 0; i < n; ++i) {
                    const double up = AT(U.data(), n, i, p), uq = AT(U.data(), n, i, q);
                    a += up * up; b += uq * uq; g += up * uq;
                }
                if (g == 0 || std::fabs(g) <= eps * std::sqrt(a * b)) continue;
                off = std::max(off, std::fabs(g) / std::sqrt(a * b));
                const double zeta = (b - a) / (2 * g);
                const double t = (zeta >= 0 ? 1.0 : -1.0) / (std::fabs(zeta) + std::sqrt(1 + zeta * zeta));
                const double cs = 1 / std::sqrt(1 + t * t), sn = cs * t;
                for (int i = 0; i < n; ++i) {
                    const double up = AT(U.data(), n, i, p), uq = AT(U.data(), n, i, q);
                    AT(U.data(), n, i, p) = cs * up - sn * uq;
                    AT(U.data(), n, i, q) = sn * up + cs * uq;
                }
            }
        if (off <= eps) break;
    }
    for (int j = 0; j < n; ++j) {
        double t = 0;
        for (int i = 0; i < n; ++i) t += AT(U.data(), n, i, j) * AT(U.data(), n, i, j);
        s[j] = std::sqrt(t);
    }
    std::sort(s, s + n, [](double a, double b) { return a > b; });
}

// gcv_function.m:33-58 on a cached H ((k+1) x k, leading dimension ldh)
double gcv_from_H(const double* H, int ldh, int k, double beta, double lambda, double trace_m) {
    const double eps = std::numeric_limits<double>::epsilon();
    std::vector<double> HtH((size_t)k * k), rhs(k), y(k);
    for (int i = 0; i < k; ++i)
        for (int j = 0; j < k; ++j) {
            double s = 0;
            for (int r = 0; r <= k; ++r) s += AT(H, ldh, r, i) * AT(H, ldh, r, j);
            AT(HtH.data(), k, i, j) = s + (i == j ? lambda : 0.0);   // :38  Hk'*Hk + lambda*eye(k)
        }
    for (int i = 0; i < k; ++i) rhs[i] = AT(H, ldh, 0, i) * beta;    // Hk'*tk, tk = beta e1
    mldivide_square(k, HtH.data(), rhs.data(), y.data());
    double rn = 0;                                                   // :40 norm(tk - Hk*yk)^2
    for (int r = 0; r <= k; ++r) {
        double t = (r == 0 ? beta : 0.0);
        double s = 0;
        for (int j = 0; j < k; ++j) s += AT(H, ldh, r, j) * y[j];
        t -= s;
        rn += t * t;
    }
    const double rnorm = std::sqrt(rn);
    const double residual_norm_sq = rnorm * rnorm;
    std::vector<double> Hs((size_t)k * k), sv(k);
    for (int j = 0; j < k; ++j)
        for (int i = 0; i < k; ++i) AT(Hs.data(), k, i, j) = AT(H, ldh, i, j);
    svd_values(k, Hs.data(), sv.data());                             // :42
    double trace_val = 0;
    for (int i = 0; i < k; ++i) trace_val += sv[i] * sv[i] / (sv[i] * sv[i] + lambda);   // :51
    const double denominator = (trace_m - trace_val) * (trace_m - trace_val);            // :52
    double g = residual_norm_sq / denominator;                                           // :54
    if (std::isnan(g) || std::isinf(g) || denominator < eps) g = 1e20;                   // :56-57
    return g;
}

// MATLAB fminbnd: golden-section search with parabolic interpolation
// (Forsythe, Malcolm & Moler, "fmin"), options TolX.
template <typename F>
double fminbnd(F f, double ax, double bx, double tolx, double* fmin_out) {
    const double c = 0.5 * (3.0 - std::sqrt(5.0));
    const double eps = std::sqrt(std::numeric_limits<double>::epsilon());
    double a = ax, b = bx;
    double v = a + c * (b - a), w = v, xf = v;
    double d = 0.0, e = 0.0;
    double fx = f(xf), fv = fx, fw = fx;
    double xm = 0.5 * (a + b);
    double tol1 = eps * std::fabs(xf) + tolx / 3.0;
    double tol2 = 2.0 * tol1;
    for (int iter = 0; iter < 500; ++iter) {
        if (std::fabs(xf - xm) <= (tol2 - 0.5 * (b - a))) break;
        int gs = 1;
        if (std::fabs(e) > tol1) {
            gs = 0;
            double r = (xf - w) * (fx - fv);
            double q = (xf - v) * (fx - fw);
            double p = (xf - v) * q - (xf - w) * r;
            q = 2.0 * (q - r);
            if (q > 0.0) p = -p;
            q = std::fabs(q);
            r = e;
            e = d;
            if (std::fabs(p) < std::fabs(0.5 * q * r) && p > q * (a - xf) && p < q * (b - xf)) {
                d = p / q;
                const double u = xf + d;
                if ((u - a) < tol2 || (b - u) < tol2) d = (xm >= xf) ? tol1 : -tol1;
            } else {
                gs = 1;
            }
        }
        if (gs) {
            e = (xf >= xm) ? a - xf : b - xf;
            d = c * e;
        }
        const double u = xf + ((d >= 0) ? 1.0 : -1.0) * std::max(std::fabs(d), tol1);
        const double fu = f(u);
        if (fu <= fx) {
            if (u >= xf) a = xf; else b = xf;
            v = w; fv = fw; w = xf; fw = fx; xf = u; fx = fu;
        } else {
            if (u < xf) a = u; else b = u;
            if (fu <= fw || w == xf) { v = w; fv = fw; w = u; fw = fu; }
            else if (fu <= fv || v == xf || v == w) { v = u; fv = fu; }
        }
        xm = 0.5 * (a + b);
        tol1 = eps * std::fabs(xf) + tolx / 3.0;
        tol2 = 2.0 * tol1;
    }
    if (fmin_out) *fmin_out = fx;
    return xf;
}

double gcv_fminbnd(const double* H, int k, double beta, double trace_m, double lo, double hi,
                   double tolx, double* gopt) {
    auto f = [&](double lam) { return gcv_from_H(H, k + 1, k, beta, lam, trace_m); };
    return fminbnd(f, lo, hi, tolx, gopt);
}

}  // namespace dense
}  // namespace hgm
