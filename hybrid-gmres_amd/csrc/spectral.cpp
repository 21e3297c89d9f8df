// Small dense host eigen-analysis for the filter-factor / perturbation bounds (outputs 5-8 of
// the four *_bounds.m files).  Everything here works on k x k or p x p projected matrices
// (k <= maxit, p = the Ritz Arnoldi length): latency-only host work, as dense.cpp.
//
// * eig_general: MATLAB/LAPACK `eig` of a real nonsymmetric matrix — Householder reduction to
//   Hessenberg form, then the Francis double-shift QR iteration with accumulated
//   transformations and back-substitution for the eigenvectors (the EISPACK orthes/hqr2
//   algorithm; no balancing).  Eigenvectors are scaled to unit 2-norm, as LAPACK dgeev does.
// * filter_factors: one iteration's phi / dphi (ABgmres_hybrid_bounds.m:42-78,
//   ABgmres_nonhybrid_bounds.m:42-73, BAgmres_hybrid_bounds.m:42-74,
//   BAgmres_nonhybrid_bounds.m:42-74).
// * ritz: the leading eigenpairs of M (A*B or B*A) from a p-step Arnoldi, replacing the dense
//   `[U,D] = eig(M)` of *_bounds.m:4-9: mu_i = Ritz values sorted by descending real part and
//   dMu_i = u_i' DeltaM u_i = y_i' (Qp' DeltaM Qp) y_i for the Ritz vector u_i = Qp y_i.
#include <algorithm>
#include <cmath>
#include <complex>
#include <limits>
#include <numeric>
#include <vector>

#include "internal.h"

namespace hgm {
namespace dense {

#define AT(M, ld, i, j) (M)[(size_t)(j) * (ld) + (i)]

namespace {

using cplx = std::complex<double>;

// Householder reduction of H (n x n, col-major, in place) to upper Hessenberg form; V receives
// the accumulated orthogonal similarity (H_in = V H V').
void hessenberg(int n, std::vector<double>& H, std::vector<double>& V) {
    std::vector<double> u(n, 0.0);
    for (int m = 1; m <= n - 2; ++m) {
        double scale = 0.0;
        for (int i = m; i < n; ++i) scale += std::fabs(AT(H.data(), n, i, m - 1));
        if (scale == 0.0) continue;
        double h = 0.0;
        for (int i = n - 1; i >= m; --i) {
            u[i] = AT(H.data(), n, i, m - 1) / scale;
            h += u[i] * u[i];
        }
        double g = std::sqrt(h);
        if (u[m] > 0) g = -g;
        h -= u[m] * g;
        u[m] -= g;
        for (int j = m; j < n; ++j) {            // H = (I - u u'/h) H
            double f = 0.0;
            for (int i = n - 1; i >= m; --i) f += u[i] * AT(H.data(), n, i, j);
            f /= h;
            for (int i = m; i < n; ++i) AT(H.data(), n, i, j) -= f * u[i];
        }
        for (int i = 0; i < n; ++i) {            // H = H (I - u u'/h)
            double f = 0.0;
            for (int j = n - 1; j >= m; --j) f += u[j] * AT(H.data(), n, i, j);
            f /= h;
            for (int j = m; j < n; ++j) AT(H.data(), n, i, j) -= f * u[j];
        }
        u[m] *= scale;
        AT(H.data(), n, m, m - 1) = scale * g;
    }
    V.assign((size_t)n * n, 0.0);
    for (int i = 0; i < n; ++i) AT(V.data(), n, i, i) = 1.0;
    for (int m = n - 2; m >= 1; --m) {
        const double hm = AT(H.data(), n, m, m - 1);
        if (hm == 0.0) continue;
        for (int i = m + 1; i < n; ++i) u[i] = AT(H.data(), n, i, m - 1);
        for (int j = m; j < n; ++j) {
            double g = 0.0;
            for (int i = m; i < n; ++i) g += u[i] * AT(V.data(), n, i, j);
            g = (g / u[m]) / hm;                  // two divisions: no underflow of u[m]*hm
            for (int i = m; i < n; ++i) AT(V.data(), n, i, j) += g * u[i];
        }
    }
    // clear the Householder vectors kept below the subdiagonal
    for (int j = 0; j < n; ++j)
        for (int i = j + 2; i < n; ++i) AT(H.data(), n, i, j) = 0.0;
}

inline cplx cdiv(double xr, double xi, double yr, double yi) { return cplx(xr, xi) / cplx(yr, yi); }

// Real Schur form of the Hessenberg H by the Francis double-shift QR iteration (V accumulates
// the transformations), eigenvalues (wr, wi), then eigenvectors by back-substitution on the
// quasi-triangular factor, transformed back with V.  Returns false when the iteration does not
// converge.  Column layout of V on return (LAPACK dgeev): a real eigenvalue j has its vector in
// column j; a complex pair (j, j+1), wi[j] > 0, has the vector of wr[j] + i wi[j] as
// V(:,j) + i V(:,j+1) and the conjugate one for j+1.
// Attribution: this routine follows the structure and variable names (exshift, norm, low/high,
// p, q, r, s, z, t, w, x, y) of the public-domain JAMA `EigenvalueDecomposition.hqr2` (NIST /
// MathWorks, 1998), itself a translation of the EISPACK routine hqr2 (Wilkinson & Reinsch,
// Handbook for Automatic Computation, Vol. II, 1971).
bool schur_vectors(int nn, std::vector<double>& Hv, std::vector<double>& Vv, double* d, double* e) {
    double* H = Hv.data();
    double* V = Vv.data();
    auto h = [&](int i, int j) -> double& { return AT(H, nn, i, j); };
    auto v = [&](int i, int j) -> double& { return AT(V, nn, i, j); };
    const double eps = std::numeric_limits<double>::epsilon();
    int n = nn - 1;
    const int low = 0, high = nn - 1;
    double exshift = 0.0, p = 0, q = 0, r = 0, s = 0, z = 0, t, w, x, y;
    double norm = 0.0;
    for (int i = 0; i < nn; ++i)
        for (int j = std::max(i - 1, 0); j < nn; ++j) norm += std::fabs(h(i, j));
    int iter = 0, total = 0;
    while (n >= low) {
        int l = n;                                           // a small subdiagonal element
        while (l > low) {
            s = std::fabs(h(l - 1, l - 1)) + std::fabs(h(l, l));
            if (s == 0.0) s = norm;
            if (std::fabs(h(l, l - 1)) < eps * s) break;
            --l;
        }
        if (l == n) {                                        // one root
            h(n, n) += exshift;
            d[n] = h(n, n);
            e[n] = 0.0;
            --n;
            iter = 0;
        } else if (l == n - 1) {                             // two roots
            w = h(n, n - 1) * h(n - 1, n);
            p = (h(n - 1, n - 1) - h(n, n)) / 2.0;
            q = p * p + w;
            z = std::sqrt(std::fabs(q));
            h(n, n) += exshift;
            h(n - 1, n - 1) += exshift;
            x = h(n, n);
            if (q >= 0) {                                    // real pair
                z = p >= 0 ? p + z : p - z;
                d[n - 1] = x + z;
                d[n] = d[n - 1];
                if (z != 0.0) d[n] = x - w / z;
                e[n - 1] = 0.0;
                e[n] = 0.0;
                x = h(n, n - 1);
                s = std::fabs(x) + std::fabs(z);
                p = x / s;
                q = z / s;
                r = std::sqrt(p * p + q * q);
                p /= r;
                q /= r;
                for (int j = n - 1; j < nn; ++j) {
                    z = h(n - 1, j);
                    h(n - 1, j) = q * z + p * h(n, j);
                    h(n, j) = q * h(n, j) - p * z;
                }
                for (int i = 0; i <= n; ++i) {
                    z = h(i, n - 1);
                    h(i, n - 1) = q * z + p * h(i, n);
                    h(i, n) = q * h(i, n) - p * z;
                }
                for (int i = low; i <= high; ++i) {
                    z = v(i, n - 1);
                    v(i, n - 1) = q * z + p * v(i, n);
                    v(i, n) = q * v(i, n) - p * z;
                }
            } else {                                         // complex pair
                d[n - 1] = x + p;
                d[n] = x + p;
                e[n - 1] = z;
                e[n] = -z;
            }
            n -= 2;
            iter = 0;
        } else {                                             // no convergence yet: shift
            if (++total > 60 * nn) return false;
            x = h(n, n);
            y = 0.0;
            w = 0.0;
            if (l < n) {
                y = h(n - 1, n - 1);
                w = h(n, n - 1) * h(n - 1, n);
            }
            if (iter == 10) {                                // exceptional shift
                exshift += x;
                for (int i = low; i <= n; ++i) h(i, i) -= x;
                s = std::fabs(h(n, n - 1)) + std::fabs(h(n - 1, n - 2));
                x = y = 0.75 * s;
                w = -0.4375 * s * s;
            }
            if (iter == 30) {                                // second exceptional shift
                s = (y - x) / 2.0;
                s = s * s + w;
                if (s > 0) {
                    s = std::sqrt(s);
                    if (y < x) s = -s;
                    s = x - w / ((y - x) / 2.0 + s);
                    for (int i = low; i <= n; ++i) h(i, i) -= s;
                    exshift += s;
                    x = y = w = 0.964;
                }
            }
            ++iter;
            int m = n - 2;                                   // two small subdiagonal elements
            while (m >= l) {
                z = h(m, m);
                r = x - z;
                s = y - z;
                p = (r * s - w) / h(m + 1, m) + h(m, m + 1);
                q = h(m + 1, m + 1) - z - r - s;
                r = h(m + 2, m + 1);
                s = std::fabs(p) + std::fabs(q) + std::fabs(r);
                p /= s;
                q /= s;
                r /= s;
                if (m == l) break;
                if (std::fabs(h(m, m - 1)) * (std::fabs(q) + std::fabs(r)) <
                    eps * (std::fabs(p) * (std::fabs(h(m - 1, m - 1)) + std::fabs(z) + std::fabs(h(m + 1, m + 1)))))
                    break;
                --m;
            }
            for (int i = m + 2; i <= n; ++i) {
                h(i, i - 2) = 0.0;
                if (i > m + 2) h(i, i - 3) = 0.0;
            }
            for (int k = m; k <= n - 1; ++k) {               // double QR step, rows l:n, cols m:n
                const bool notlast = (k != n - 1);
                if (k != m) {
                    p = h(k, k - 1);
                    q = h(k + 1, k - 1);
                    r = notlast ? h(k + 2, k - 1) : 0.0;
                    x = std::fabs(p) + std::fabs(q) + std::fabs(r);
                    if (x == 0.0) continue;
                    p /= x;
                    q /= x;
                    r /= x;
                }
                s = std::sqrt(p * p + q * q + r * r);
                if (p < 0) s = -s;
                if (s == 0) continue;
                if (k != m) h(k, k - 1) = -s * x;
                else if (l != m) h(k, k - 1) = -h(k, k - 1);
                p += s;
                x = p / s;
                y = q / s;
                z = r / s;
                q /= p;
                r /= p;
                for (int j = k; j < nn; ++j) {
                    p = h(k, j) + q * h(k + 1, j);
                    if (notlast) {
                        p += r * h(k + 2, j);
                        h(k + 2, j) -= p * z;
                    }
                    h(k, j) -= p * x;
                    h(k + 1, j) -= p * y;
                }
                for (int i = 0; i <= std::min(n, k + 3); ++i) {
                    p = x * h(i, k) + y * h(i, k + 1);
                    if (notlast) {
                        p += z * h(i, k + 2);
                        h(i, k + 2) -= p * r;
                    }
                    h(i, k) -= p;
                    h(i, k + 1) -= p * q;
                }
                for (int i = low; i <= high; ++i) {
                    p = x * v(i, k) + y * v(i, k + 1);
                    if (notlast) {
                        p += z * v(i, k + 2);
                        v(i, k + 2) -= p * r;
                    }
                    v(i, k) -= p;
                    v(i, k + 1) -= p * q;
                }
            }
        }
    }
    if (norm == 0.0) return true;
    // back-substitution: eigenvectors of the quasi-triangular factor
    for (n = nn - 1; n >= 0; --n) {
        p = d[n];
        q = e[n];
        if (q == 0) {                                        // real vector
            int l = n;
            h(n, n) = 1.0;
            for (int i = n - 1; i >= 0; --i) {
                w = h(i, i) - p;
                r = 0.0;
                for (int j = l; j <= n; ++j) r += h(i, j) * h(j, n);
                if (e[i] < 0.0) {
                    z = w;
                    s = r;
                } else {
                    l = i;
                    if (e[i] == 0.0) {
                        h(i, n) = w != 0.0 ? -r / w : -r / (eps * norm);
                    } else {                                 // 2 x 2 real block
                        x = h(i, i + 1);
                        y = h(i + 1, i);
                        q = (d[i] - p) * (d[i] - p) + e[i] * e[i];
                        t = (x * s - z * r) / q;
                        h(i, n) = t;
                        h(i + 1, n) = std::fabs(x) > std::fabs(z) ? (-r - w * t) / x : (-s - y * t) / z;
                    }
                    t = std::fabs(h(i, n));
                    if ((eps * t) * t > 1)
                        for (int j = i; j <= n; ++j) h(j, n) /= t;
                }
            }
        } else if (q < 0) {                                  // complex vector (second of a pair)
            int l = n - 1;
            if (std::fabs(h(n, n - 1)) > std::fabs(h(n - 1, n))) {
                h(n - 1, n - 1) = q / h(n, n - 1);
                h(n - 1, n) = -(h(n, n) - p) / h(n, n - 1);
            } else {
                const cplx cd = cdiv(0.0, -h(n - 1, n), h(n - 1, n - 1) - p, q);
                h(n - 1, n - 1) = cd.real();
                h(n - 1, n) = cd.imag();
            }
            h(n, n - 1) = 0.0;
            h(n, n) = 1.0;
            for (int i = n - 2; i >= 0; --i) {
                double ra = 0.0, sa = 0.0, vr, vi;
                for (int j = l; j <= n; ++j) {
                    ra += h(i, j) * h(j, n - 1);
                    sa += h(i, j) * h(j, n);
                }
                w = h(i, i) - p;
                if (e[i] < 0.0) {
                    z = w;
                    r = ra;
                    s = sa;
                } else {
                    l = i;
                    if (e[i] == 0) {
                        const cplx cd = cdiv(-ra, -sa, w, q);
                        h(i, n - 1) = cd.real();
                        h(i, n) = cd.imag();
                    } else {
                        x = h(i, i + 1);
                        y = h(i + 1, i);
                        vr = (d[i] - p) * (d[i] - p) + e[i] * e[i] - q * q;
                        vi = (d[i] - p) * 2.0 * q;
                        if (vr == 0.0 && vi == 0.0)
                            vr = eps * norm * (std::fabs(w) + std::fabs(q) + std::fabs(x) + std::fabs(y) + std::fabs(z));
                        const cplx cd = cdiv(x * r - z * ra + q * sa, x * s - z * sa - q * ra, vr, vi);
                        h(i, n - 1) = cd.real();
                        h(i, n) = cd.imag();
                        if (std::fabs(x) > (std::fabs(z) + std::fabs(q))) {
                            h(i + 1, n - 1) = (-ra - w * h(i, n - 1) + q * h(i, n)) / x;
                            h(i + 1, n) = (-sa - w * h(i, n) - q * h(i, n - 1)) / x;
                        } else {
                            const cplx c2 = cdiv(-r - y * h(i, n - 1), -s - y * h(i, n), z, q);
                            h(i + 1, n - 1) = c2.real();
                            h(i + 1, n) = c2.imag();
                        }
                    }
                    t = std::max(std::fabs(h(i, n - 1)), std::fabs(h(i, n)));
                    if ((eps * t) * t > 1)
                        for (int j = i; j <= n; ++j) {
                            h(j, n - 1) /= t;
                            h(j, n) /= t;
                        }
                }
            }
        }
    }
    // back-transformation: eigenvectors of the input matrix
    for (int j = nn - 1; j >= low; --j)
        for (int i = low; i <= high; ++i) {
            z = 0.0;
            for (int k = low; k <= std::min(j, high); ++k) z += v(i, k) * h(k, j);
            v(i, j) = z;
        }
    return true;
}

// The eigenvector of eigenvalue j as complex numbers (dgeev layout, see schur_vectors).
std::vector<cplx> eigvec(int n, const double* V, const double* wi, int j) {
    std::vector<cplx> u(n);
    if (wi[j] == 0.0) {
        for (int i = 0; i < n; ++i) u[i] = AT(V, n, i, j);
    } else if (wi[j] > 0.0) {
        for (int i = 0; i < n; ++i) u[i] = cplx(AT(V, n, i, j), AT(V, n, i, j + 1));
    } else {
        for (int i = 0; i < n; ++i) u[i] = cplx(AT(V, n, i, j - 1), -AT(V, n, i, j));
    }
    return u;
}

// stable sort of the indices by the real parts (ascending, or descending as MATLAB's
// sort(...,'descend'), which keeps equal elements in their original order)
std::vector<int> sort_real(int n, const double* wr, bool descend) {
    std::vector<int> o(n);
    std::iota(o.begin(), o.end(), 0);
    if (descend) std::stable_sort(o.begin(), o.end(), [&](int a, int b) { return wr[a] > wr[b]; });
    else std::stable_sort(o.begin(), o.end(), [&](int a, int b) { return wr[a] < wr[b]; });
    return o;
}

}  // namespace

bool eig_general(int n, const double* A, double* wr, double* wi, double* Vout) {
    if (n <= 0) return true;
    std::vector<double> H(A, A + (size_t)n * n), V;
    hessenberg(n, H, V);
    if (!schur_vectors(n, H, V, wr, wi)) return false;
    // unit 2-norm eigenvectors (complex pairs: the norm of the complex vector), as dgeev
    for (int j = 0; j < n; ++j) {
        if (wi[j] == 0.0) {
            double s = 0;
            for (int i = 0; i < n; ++i) s += AT(V.data(), n, i, j) * AT(V.data(), n, i, j);
            s = std::sqrt(s);
            if (s > 0)
                for (int i = 0; i < n; ++i) AT(V.data(), n, i, j) /= s;
        } else if (wi[j] > 0.0 && j + 1 < n) {
            double s = 0;
            for (int i = 0; i < n; ++i)
                s += AT(V.data(), n, i, j) * AT(V.data(), n, i, j) + AT(V.data(), n, i, j + 1) * AT(V.data(), n, i, j + 1);
            s = std::sqrt(s);
            if (s > 0)
                for (int i = 0; i < n; ++i) {
                    AT(V.data(), n, i, j) /= s;
                    AT(V.data(), n, i, j + 1) /= s;
                }
            ++j;
        }
    }
    if (Vout) std::copy(V.begin(), V.end(), Vout);
    return true;
}

void filter_factors(const double* H, int ldh, int k, const double* dK, int lddk, const double* mu,
                    const double* dmu, double lambda, int side, int hybrid, double* phi, double* dphi) {
    const double eps0 = std::numeric_limits<double>::epsilon();   // eps0_current = eps
    std::vector<double> P((size_t)k * k);
    if (side == HGM_SIDE_BA && hybrid) {
        // [W, Th] = eig(Hk_full'*Hk_full, Hk_small)   (BAgmres_hybrid_bounds.m:44-46), as the
        // standard problem of Hk_small \ (Hk_full'*Hk_full): same eigenpairs when Hk_small is
        // nonsingular (the Arnoldi stopped before any breakdown)
        std::vector<double> G((size_t)k * k), Hs((size_t)k * k), col(k), sol(k);
        for (int i = 0; i < k; ++i)
            for (int j = 0; j < k; ++j) {
                double s = 0;
                for (int r = 0; r <= k; ++r) s += AT(H, ldh, r, i) * AT(H, ldh, r, j);
                AT(G.data(), k, i, j) = s;
            }
        for (int j = 0; j < k; ++j)
            for (int i = 0; i < k; ++i) AT(Hs.data(), k, i, j) = AT(H, ldh, i, j);
        for (int j = 0; j < k; ++j) {
            for (int i = 0; i < k; ++i) col[i] = AT(G.data(), k, i, j);
            mldivide_square(k, Hs.data(), col.data(), sol.data());
            for (int i = 0; i < k; ++i) AT(P.data(), k, i, j) = sol[i];
        }
    } else {
        // P = Hk_small + H(k+1,k)^2 * (Hk_small' \ (ek*ek'))   (AB :48 / nonhybrid :48 / :47):
        // the right-hand side is zero except its last column, so only column k changes
        std::vector<double> HsT((size_t)k * k), ek(k, 0.0), xk(k);
        for (int j = 0; j < k; ++j)
            for (int i = 0; i < k; ++i) {
                AT(P.data(), k, i, j) = AT(H, ldh, i, j);
                AT(HsT.data(), k, j, i) = AT(H, ldh, i, j);
            }
        ek[k - 1] = 1.0;
        mldivide_square(k, HsT.data(), ek.data(), xk.data());
        const double hk = AT(H, ldh, k, k - 1);
        const double h2 = hk * hk;
        for (int i = 0; i < k; ++i) AT(P.data(), k, i, k - 1) = AT(P.data(), k, i, k - 1) + h2 * xk[i];
        if (hybrid)                                                   // P_reg = P_unreg + lambda*eye(k) (AB :49)
            for (int i = 0; i < k; ++i) AT(P.data(), k, i, i) = AT(P.data(), k, i, i) + lambda;
    }
    std::vector<double> wr(k), wi(k), W((size_t)k * k);
    if (!eig_general(k, P.data(), wr.data(), wi.data(), W.data()))
        throw Error{HGM_E_ARG, "filter factors: the QR iteration did not converge"};
    const std::vector<int> o = sort_real(k, wr.data(), false);      // [Theta, p_sort] = sort(Theta)
    std::vector<double> Th(k), dTh(k);
    for (int j = 0; j < k; ++j) {
        Th[j] = wr[o[j]];
        // dTheta = real(diag(W' * dK * W))  (conjugate transpose)
        const std::vector<cplx> w = eigvec(k, W.data(), wi.data(), o[j]);
        cplx acc = 0;
        for (int a = 0; a < k; ++a) {
            cplx t = 0;
            for (int b = 0; b < k; ++b) t += AT(dK, lddk, a, b) * w[b];
            acc += std::conj(w[a]) * t;
        }
        dTh[j] = acc.real();
    }
    // Clog(i) = sum(log(max(1 - s2l(i)./Theta.', eps0)))  and the products without factor j
    std::vector<double> logd((size_t)k * k);
    for (int i = 0; i < k; ++i) {
        const double s2l = hybrid ? mu[i] + lambda : mu[i];
        double clog = 0;
        for (int j = 0; j < k; ++j) {
            const double lj = std::log(std::max(1.0 - s2l / Th[j], eps0));
            logd[(size_t)i * k + j] = lj;
            clog += lj;
        }
        const double pfin = std::exp(clog);
        double s1 = 0, s2 = 0;
        for (int j = 0; j < k; ++j) {
            const double pex = std::exp(clog - logd[(size_t)i * k + j]);   // P_excl(i,j)
            s1 += (dTh[j] / (Th[j] * Th[j])) * pex;
            s2 += (1.0 / Th[j]) * pex;
        }
        if (hybrid) {
            phi[i] = (mu[i] / s2l) * (1.0 - pfin);
            const double t1 = -mu[i] * s1;
            const double t2 = (lambda / (s2l * s2l)) * (1.0 - pfin) * dmu[i];
            const double t3 = (mu[i] / s2l) * s2 * dmu[i];
            dphi[i] = t1 + t2 + t3;
        } else {
            phi[i] = 1.0 - pfin;
            dphi[i] = -mu[i] * s1 + s2 * dmu[i];
        }
    }
}

void ritz(const double* Hp, int ldh, int p, double h_next, const double* G, int ldg, int nev, double* mu,
          double* dmu, double* resid) {
    std::vector<double> Hs((size_t)p * p), wr(p), wi(p), Y((size_t)p * p);
    for (int j = 0; j < p; ++j)
        for (int i = 0; i < p; ++i) AT(Hs.data(), p, i, j) = AT(Hp, ldh, i, j);
    if (!eig_general(p, Hs.data(), wr.data(), wi.data(), Y.data()))
        throw Error{HGM_E_ARG, "Ritz values: the QR iteration did not converge"};
    const std::vector<int> o = sort_real(p, wr.data(), true);        // sort(mu_full, 'descend')
    for (int i = 0; i < nev && i < p; ++i) {
        const int j = o[i];
        mu[i] = wr[j];                                                // mu_full = real(diag(D_M))
        const std::vector<cplx> y = eigvec(p, Y.data(), wi.data(), j);
        // dMu = u' DeltaM u for u = Qp y: y.' G y for a real pair (the reference's non-conjugated
        // sum(UA .* (DeltaM*UA))); for a complex pair the phase-invariant Re(y^H G y)
        cplx acc = 0;
        for (int a = 0; a < p; ++a) {
            cplx t = 0;
            for (int b = 0; b < p; ++b) t += AT(G, ldg, a, b) * y[b];
            acc += (wi[j] == 0.0 ? y[a] : std::conj(y[a])) * t;
        }
        dmu[i] = acc.real();
        if (resid) resid[i] = std::fabs(h_next) * std::abs(y[p - 1]);   // ||M u - mu u|| (Arnoldi relation)
    }
}

}  // namespace dense
}  // namespace hgm
