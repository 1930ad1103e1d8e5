/* Sanitizer driver for the oracle (ASan + UBSan build, `make -C oracle sanitize`; TEST INFRASTRUCTURE ONLY, see
 * mmpc_oracle.h): every solve variant (Gauss-Newton, exact Hessian, control bounds, state bounds, linear mode,
 * exo), the NLP evaluators and the generators on small batches, including non-finite inputs and N = 1.  The
 * sanitizers turn any out-of-bounds access, leak or undefined behaviour into a non-zero exit. */
#include <math.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "mmpc_oracle.h"

static int run(int model, int N, int B, int hess, int bounded, int xbounded, int linear) {
    const int nx = model == ORACLE_MODEL_EXO_ARM ? 8 : 4, nu = model == ORACLE_MODEL_EXO_ARM ? 4 : 2;
    const int NV = nx * (N + 1) + nu * N;
    double* x0 = calloc((size_t)B * nx, sizeof(double));
    double* up = calloc((size_t)B * nu, sizeof(double));
    double* tr = calloc((size_t)B * N * nx, sizeof(double));
    double* V = calloc((size_t)B * NV, sizeof(double));
    double* kkt = calloc((size_t)B, sizeof(double));
    double* J = calloc((size_t)B, sizeof(double));
    double* g = calloc((size_t)N * nx, sizeof(double));
    double* hb = calloc((size_t)N * (nx + nu) * (nx + nu), sizeof(double));
    int32_t* st = calloc((size_t)B, sizeof(int32_t));
    int32_t* it = calloc((size_t)B, sizeof(int32_t));
    double w[48], ul[16], uu[16], xl[16], xu[16];
    for (int i = 0; i < nx; ++i) { w[i] = 10.0; xl[i] = i >= nx / 2 ? -2.0 : -1e20; xu[i] = i >= nx / 2 ? 2.0 : 1e20; }
    for (int i = 0; i < nu; ++i) { w[nx + i] = 1.0; w[nx + nu + i] = 0.01; ul[i] = -3.0; uu[i] = 3.0; }
    if (model == ORACLE_MODEL_EXO_ARM) oracle_synth_exo(7, 0, B, N, 0.002, x0, up, tr);
    else oracle_synth_two_link(7, 0, B, N, 0.002, x0, up, tr);
    if (B > 2) { x0[nx] = NAN; tr[2 * N * nx + 1] = INFINITY; }  /* non-finite inputs: status 3, no UB */
    oracle_set_hessian(hess);
    int rc = oracle_solve_batch_xb(model, linear, N, 0.002, B, x0, up, tr, w, 0, bounded ? ul : NULL,
                                   bounded ? uu : NULL, xbounded ? xl : NULL, xbounded ? xu : NULL, 30, 1e-8, 1e-10, V,
                                   st, it, kkt, J, 1);
    oracle_set_hessian(ORACLE_HESS_GAUSS_NEWTON);
    oracle_nlp_eval(model, N, 0.002, V, up, tr, w, J, g);
    if (oracle_nlp_hess(model, N, 0.002, V, up, tr, w, 1.0, g, hb) != 0 && model == ORACLE_MODEL_TWO_LINK_ARM) rc = -2;
    if (N > 1) {
        double* U = calloc((size_t)N * nu, sizeof(double));
        double* gr = calloc((size_t)N * nu, sizeof(double));
        oracle_reduced_gradient(model, N, 0.002, x0, U, up, tr, w, gr);
        free(U);
        free(gr);
    }
    int conv = 0;
    for (int b = 0; b < B; ++b) conv += st[b] == 0;
    printf("model %d N %d B %d hess %d bounds %d/%d linear %d: rc %d, %d converged\n", model, N, B, hess, bounded,
           xbounded, linear, rc, conv);
    free(x0); free(up); free(tr); free(V); free(kkt); free(J); free(g); free(hb); free(st); free(it);
    return rc;
}

int main(void) {
    int bad = 0;
    bad |= run(ORACLE_MODEL_TWO_LINK_ARM, 30, 6, ORACLE_HESS_GAUSS_NEWTON, 0, 0, 0);
    bad |= run(ORACLE_MODEL_TWO_LINK_ARM, 30, 6, ORACLE_HESS_EXACT, 0, 0, 0);
    bad |= run(ORACLE_MODEL_TWO_LINK_ARM, 1, 3, ORACLE_HESS_EXACT, 0, 0, 0);
    bad |= run(ORACLE_MODEL_TWO_LINK_ARM, 20, 4, ORACLE_HESS_GAUSS_NEWTON, 1, 0, 0);
    bad |= run(ORACLE_MODEL_TWO_LINK_ARM, 20, 4, ORACLE_HESS_GAUSS_NEWTON, 1, 1, 0);
    bad |= run(ORACLE_MODEL_TWO_LINK_ARM, 20, 4, ORACLE_HESS_EXACT, 0, 0, 1);
    bad |= run(ORACLE_MODEL_EXO_ARM, 12, 4, ORACLE_HESS_GAUSS_NEWTON, 0, 0, 0);
    bad |= run(ORACLE_MODEL_EXO_ARM, 12, 3, ORACLE_HESS_GAUSS_NEWTON, 1, 1, 0);
    if (bad) { fprintf(stderr, "oracle sanitize check failed\n"); return 1; }
    printf("oracle sanitize ok\n");
    return 0;
}
