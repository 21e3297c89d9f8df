// Filter-factor / perturbation bounds at scale: outputs 5-8 (phi_final, dphi_final, phi_iter,
// dphi_iter) of ABgmres_hybrid_bounds.m, ABgmres_nonhybrid_bounds.m, BAgmres_hybrid_bounds.m
// and BAgmres_nonhybrid_bounds.m.
//
// The reference forms M = A*B (or B*A) densely and calls `[U, D] = eig(M)` (*_bounds.m:4-9):
// O(dim^3) time and O(dim^2) memory, infeasible past dim ~ 1e4.  Only the k <= maxit leading
// eigenpairs are ever used (mu_full(1:k), UA(:,1:k) at :55-58), so here they are Ritz pairs
// of a p-step Arnoldi on M, run on the device with classical Gram-Schmidt twice (the full
// reorthogonalisation eigenvalue accuracy needs).  With p = dim the Arnoldi spans the whole
// space and the Ritz pairs are the eigenpairs of M to rounding: that is the parity setting of
// the tests.  Everything else is the reference's own sequence on the solve's Krylov basis:
//   dK = Qk' * DeltaM * Qk                        (AB :44, BA :43)  -> device SpMVs + dots
//   P  = Hk + H(k+1,k)^2 (Hk' \ ek ek') (+ lambda I) / eig(H'H, Hk)   -> spectral.cpp
//   dMu_i = u_i' DeltaM u_i = y_i' (Qp' DeltaM Qp) y_i                -> spectral.cpp
// DeltaM is passed as a device operator, or as the product of two (DeltaM = L * R, e.g. the
// reference's A*E / E*A with E = B - A', analyze_regularization.m:12-15), applied to vectors
// and never formed.
#include <algorithm>
#include <cmath>
#include <cstring>
#include <vector>

#include "internal.h"

namespace hgm {

// solvers.cpp
struct GmresSpec {
    int side;
    int proj;
    bool lambda_in_op;
    bool x_preassigned;
};
int gmres_family(hgm_ctx* c, const GmresSpec& sp, const hgm_opts* o, const hgm_mat* A, const hgm_mat* B,
                 const double* b_in, const double* xt_in, double tol, int maxit, double lambda, double* x_out,
                 double* err_out, double* res_out, int* niters);

namespace {

enum { PROJ_LS = 0, PROJ_PTR = 1 };

inline int64_t round64(int64_t x) { return (x + 63) / 64 * 64; }

// ritz_steps = 0 runs the full Arnoldi (p = dim, the eigenpairs of M) up to this dimension
constexpr int64_t kRitzFullDim = 1024;

struct DeltaM {
    const hgm_mat* L;
    const hgm_mat* R;   // nullptr: DeltaM = L
    // y = DeltaM x (dim-vectors in the Krylov space's stored order)
    void apply(hgm_ctx* c, const double* x, double* y) const {
        if (R) {
            double* t = c->buf<double>("fb_dm_t", R->rows + 1);
            spmv<double>(c, R, x, t, EPI_NONE, 0.0, nullptr, KC_SPMV_A);
            spmv<double>(c, L, t, y, EPI_NONE, 0.0, nullptr, KC_SPMV_B);
        } else {
            spmv<double>(c, L, x, y, EPI_NONE, 0.0, nullptr, KC_SPMV_A);
        }
    }
};

// G = Qb(:,0:cnt-1)' * DeltaM * Qb(:,0:cnt-1) (cnt x cnt, column-major, host)
std::vector<double> projected_delta(hgm_ctx* c, const DeltaM& dm, const double* Qb, int64_t ldq, int64_t dim,
                                    int cnt) {
    const int64_t ldw = round64(dim);
    double* W = c->buf<double>("fb_W", (size_t)ldw * cnt);
    double* Gd = c->buf<double>("fb_G", (size_t)cnt * cnt);
    for (int j = 0; j < cnt; ++j) dm.apply(c, Qb + (int64_t)j * ldq, W + (int64_t)j * ldw);
    for (int j = 0; j < cnt; ++j) multidot<double>(c, dim, cnt, Qb, ldq, W + (int64_t)j * ldw, Gd + (size_t)j * cnt);
    std::vector<double> G((size_t)cnt * cnt);
    Reader rd(c);
    rd.add(G.data(), Gd, sizeof(double) * G.size());
    rd.go();
    return G;
}

}  // namespace

int gmres_bounds_filter(hgm_ctx* c, const hgm_opts* o, const hgm_mat* A, const hgm_mat* B, const double* b,
                        const double* xt, double tol, int maxit, double lambda, int side, int hybrid,
                        const hgm_mat* dML, const hgm_mat* dMR, int ritz_steps, double* x_out, double* err_out,
                        double* res_out, int* niters, double* phi, double* dphi, double* mu_out, double* ritz_res) {
    solver_guard(c);
    HGM_REQUIRE(A != nullptr && B != nullptr, "A and B are required");
    HGM_REQUIRE(c->world == 1, "filter-factor bounds: single rank");
    HGM_REQUIRE(dML != nullptr, "DeltaM is required");
    HGM_REQUIRE(maxit >= 1, "maxit must be >= 1");
    const bool nspace = side == HGM_SIDE_BA;
    const int64_t dim = nspace ? A->cols : A->rows;
    const PixOrder ord = nspace ? A->col_order : PixOrder{};
    if (dMR) {
        HGM_REQUIRE(dMR->cols == dim && dML->rows == dim && dML->cols == dMR->rows,
                    "DeltaM = L*R must be dim x dim (AB: m x m, BA: n x n)");
        HGM_REQUIRE(dMR->dtype == HGM_F64, "DeltaM is fp64");
        HGM_REQUIRE(dMR->col_order == ord && dML->col_order == dMR->row_order,
                    "DeltaM's factors must share the Krylov space's stored order");
    } else {
        HGM_REQUIRE(dML->rows == dim && dML->cols == dim, "DeltaM must be dim x dim (AB: m x m, BA: n x n)");
        HGM_REQUIRE(dML->col_order == ord, "DeltaM must share the Krylov space's stored order");
    }
    HGM_REQUIRE(dML->dtype == HGM_F64, "DeltaM is fp64");
    HGM_REQUIRE(dML->row_order == ord, "DeltaM must share the Krylov space's stored order");
    const DeltaM dm{dML, dMR};

    // ---- outputs 1-4: the solve itself (*_bounds.m:11-41), keeping H and the basis ----
    hgm_opts o2{0, HGM_MGS, nullptr};
    if (o) o2 = *o;
    std::vector<double> H((size_t)(maxit + 1) * maxit, 0.0);
    o2.H_out = H.data();
    int k = 0;
    int st = gmres_family(c, GmresSpec{side, hybrid ? PROJ_PTR : PROJ_LS, false, false}, &o2, A, B, b, xt, tol, maxit,
                          hybrid ? lambda : 0.0, x_out, err_out, res_out, &k);
    if (st != HGM_OK) return st;
    if (o && o->H_out) std::memcpy(o->H_out, H.data(), sizeof(double) * H.size());
    if (niters) *niters = k;
    auto Hh = [&](int i, int j) { return H[(size_t)j * (maxit + 1) + i]; };
    // a breakdown at iteration k (H(k+1,k) == 0) leaves phi_iter{k} unassigned in the
    // reference (the loop breaks at :31 before :80): that column is NaN here
    const bool broke = Hh(k, k - 1) == 0.0;
    const int kf = broke ? k - 1 : k;

    // the solve's basis Q(:,0:k), read with gmres_family's own leading dimension: an n-space basis
    // on a communicator (a one-rank RCCL context included) is laid out for the sharded path
    const int64_t ldq = krylov_ld(c, dim, nspace && (c->world > 1 || c->nccl != nullptr));
    const double* Q = c->buf<double>("Q", (size_t)ldq * (maxit + 1));
    // ---- dK = Qk' * DeltaM * Qk for every k at once (the leading blocks of the final one) ----
    const std::vector<double> dK = kf > 0 ? projected_delta(c, dm, Q, ldq, dim, kf) : std::vector<double>();

    // ---- leading eigenpairs of M: p-step Arnoldi with CGS2 (replaces eig(M), :4-9) ----
    // default: p = dim (eig(M) itself, to rounding) wherever that is cheap -- the reference's own
    // problems (n = 32 shaw/heat/deriv2, 32^2 phantoms) -- else max(2k+10, 20) Ritz steps
    int p = ritz_steps > 0 ? ritz_steps : (dim <= kRitzFullDim ? (int)dim : std::max(2 * kf + 10, 20));
    p = (int)std::min<int64_t>(std::max(p, kf), dim);
    std::vector<double> mu(std::max(kf, 1)), dmu(std::max(kf, 1)), rres(std::max(kf, 1));
    if (kf > 0) {
        const int64_t ldp = krylov_ld(c, dim, false);
        double* Qp = c->buf<double>("fb_Qp", (size_t)ldp * (p + 1));
        if (krylov_padded(c, ldp)) HGM_HIP(hipMemsetAsync(Qp, 0, sizeof(double) * ldp * (p + 1), c->stream));
        double* Hd = c->buf<double>("fb_H", (size_t)(p + 1) * p + 8);
        double* hsink = c->buf<double>("fb_hsink", (size_t)p + 8);
        double* tm = c->buf<double>("fb_t", std::max(A->rows, A->cols) + 1);
        double* nrm = c->buf<double>("fb_nrm", 2);
        HGM_HIP(hipMemsetAsync(Hd, 0, sizeof(double) * ((size_t)(p + 1) * p + 8), c->stream));
        const FusedPlan* fplan = nspace ? nullptr : fused_ab_plan(c, A, B);
        const uint64_t seed = 0x5EEDB0A4D5ull;
        fill_hash<double>(c, dim, Qp, seed);
        normalize_to<double>(c, dim, Qp, nrm);
        std::vector<double> Hp((size_t)(p + 1) * p, 0.0);
        double hmax = 0.0;
        // The steps are enqueued back to back and their H columns read once; the scan then applies
        // the per-step breakdown test with the running max.  After an invariant subspace at step j
        // (rare) the fresh vector is made and the steps from j+1 are enqueued again, so the result is
        // that of a per-step test.
        int j0 = 0;
        while (j0 < p) {
            for (int j = j0; j < p; ++j) {
                const double* qj = Qp + (int64_t)j * ldp;
                double* v = Qp + (int64_t)(j + 1) * ldp;
                if (nspace) {                                    // M = B*A
                    spmv<double>(c, A, qj, tm, EPI_NONE, 0.0, nullptr, KC_SPMV_A);
                    spmv<double>(c, B, tm, v, EPI_NONE, 0.0, nullptr, KC_SPMV_B);
                } else if (fplan) {                              // M = A*B, one pass over B
                    fused_ab(c, B, fplan, qj, tm, v);
                } else {                                         // M = A*B
                    spmv<double>(c, B, qj, tm, EPI_NONE, 0.0, nullptr, KC_SPMV_B);
                    spmv<double>(c, A, tm, v, EPI_NONE, 0.0, nullptr, KC_SPMV_A);
                }
                cgs2<double>(c, dim, Qp, ldp, j, Hd + (size_t)j * (p + 1), false);
            }
            Reader rd(c);
            rd.add(&Hp[(size_t)j0 * (p + 1)], Hd + (size_t)j0 * (p + 1), sizeof(double) * (size_t)(p - j0) * (p + 1));
            rd.go();
            int restart = p;
            for (int j = j0; j < p; ++j) {
                for (int i = 0; i < j + 2; ++i) hmax = std::max(hmax, std::fabs(Hp[(size_t)j * (p + 1) + i]));
                for (int i = j + 2; i <= p; ++i) Hp[(size_t)j * (p + 1) + i] = 0.0;
                double& hsub = Hp[(size_t)j * (p + 1) + j + 1];
                if (j + 1 < p && !(hsub > 1e-12 * hmax)) {
                    // invariant subspace found: continue from a fresh vector orthogonal to it
                    // (H(j+1,j) = 0 keeps Hp block upper triangular, so its eigenvalues stay M's)
                    hsub = 0.0;
                    double* v = Qp + (int64_t)(j + 1) * ldp;
                    fill_hash<double>(c, dim, v, seed + 0x1000 + (uint64_t)j);
                    cgs2<double>(c, dim, Qp, ldp, j, hsink, false);
                    restart = j + 1;
                    break;
                }
            }
            j0 = restart;
        }
        const double h_next = Hp[(size_t)(p - 1) * (p + 1) + p];
        const std::vector<double> G = projected_delta(c, dm, Qp, ldp, dim, p);
        dense::ritz(Hp.data(), p + 1, p, h_next, G.data(), p, kf, mu.data(), dmu.data(), rres.data());
    }

    // ---- phi / dphi per iteration (*_bounds.m:42-81) ----
    const double nan = std::nan("");
    if (phi) std::fill(phi, phi + (size_t)maxit * maxit, 0.0);
    if (dphi) std::fill(dphi, dphi + (size_t)maxit * maxit, 0.0);
    std::vector<double> ph(std::max(kf, 1)), dph(std::max(kf, 1));
    for (int kk = 1; kk <= kf; ++kk) {
        dense::filter_factors(H.data(), maxit + 1, kk, dK.data(), kf, mu.data(), dmu.data(), lambda, side, hybrid,
                              ph.data(), dph.data());
        if (phi) std::memcpy(phi + (size_t)(kk - 1) * maxit, ph.data(), sizeof(double) * kk);
        if (dphi) std::memcpy(dphi + (size_t)(kk - 1) * maxit, dph.data(), sizeof(double) * kk);
    }
    if (broke) {
        if (phi) std::fill(phi + (size_t)(k - 1) * maxit, phi + (size_t)(k - 1) * maxit + k, nan);
        if (dphi) std::fill(dphi + (size_t)(k - 1) * maxit, dphi + (size_t)(k - 1) * maxit + k, nan);
    }
    if (mu_out) std::memcpy(mu_out, mu.data(), sizeof(double) * kf);
    if (ritz_res) std::memcpy(ritz_res, rres.data(), sizeof(double) * kf);
    return HGM_OK;
}

}  // namespace hgm
