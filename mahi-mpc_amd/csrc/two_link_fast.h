// two_link_fast.h -- the 2-link arm of examples/ex_model_generate.cpp:24-43 (L = m = 1, g = 9.81) with its first
// and second derivatives written out by hand for the GPU.  The two acceleration numerators of :36-37, grouped by
// their monomials in (dA, dB, TA, TB) with coefficients in the link angles (E = 1 + cos qB, F = 3 + 2 cos qB):
//   nA = TA - E TB + sB (dA + dB)^2 + cB sB dA^2 + g (cB cAB - 2 cA)
//   nB = E TA - F TB + sB (F dA^2 + E dB^2 + 2 E dA dB) + g ((2 + cB) cAB - 2 E cA)
//   qA_ddot = -nA / D,  qB_ddot = nB / D,  D = cB^2 - 2   (cAB = cos(qA + qB) = cA cB - sA sB)
// so one sincos per angle replaces the three trigonometric calls of the term-by-term form, and the Jacobian and
// the weighted Hessian W = sum_s lam_s d^2 a_s / d(x,u)^2 follow from the quotient rule with D depending on qB only.
// Compiled for the device (models.h, TwoLinkArm) and for the host by the tests (oracle/builtin_hess_host.cpp), which
// check it against the oracle's independent dual / hyper-dual restatement term by term of :36-37.
#pragma once
#include "fast_trig.h"

namespace mmpc {

struct TwoLinkFast {
    static constexpr double kG = 9.81;
    struct Terms {
        double sA, cA, sB, cB, sAB, cAB, E, F, iD, nA, nB;
    };
    MMPC_HD static void terms(const double* x, const double* u, Terms& t) {
        const trig_cptr TK = trig_table();
        sincos_fast(TK, x[0], &t.sA, &t.cA);
        sincos_fast(TK, x[1], &t.sB, &t.cB);
        t.cAB = fma(t.cA, t.cB, -t.sA * t.sB);
        t.sAB = fma(t.sA, t.cB, t.cA * t.sB);
        t.E = 1.0 + t.cB;
        t.F = fma(2.0, t.cB, 3.0);
        t.iD = 1.0 / fma(t.cB, t.cB, -2.0);
        const double dA = x[2], dB = x[3], TA = u[0], TB = u[1], dS = dA + dB;
        t.nA = fma(-t.E, TB, TA) + t.sB * fma(dS, dS, t.cB * dA * dA) + kG * fma(t.cB, t.cAB, -2.0 * t.cA);
        t.nB = fma(t.E, TA, -t.F * TB) + t.sB * fma(t.F * dA, dA, t.E * dB * fma(2.0, dA, dB)) +
               kG * fma(2.0 + t.cB, t.cAB, -2.0 * t.E * t.cA);
    }
    MMPC_HD static void eval(const double* x, const double* u, double* xd) {
        Terms t;
        terms(x, u, t);
        xd[0] = x[2];
        xd[1] = x[3];
        xd[2] = -t.nA * t.iD;
        xd[3] = t.nB * t.iD;
    }
    // gradients of nA, nB over (qA, qB, dA, dB, TA, TB)
    MMPC_HD static void grads(const double* x, const double* u, const Terms& t, double* gA, double* gB) {
        const double dA = x[2], dB = x[3], TA = u[0], TB = u[1], dS = dA + dB;
        const double c2s2 = fma(t.cB, t.cB, -t.sB * t.sB);   // d(cB sB)/dqB
        gA[0] = kG * fma(-t.cB, t.sAB, 2.0 * t.sA);
        gA[1] = t.sB * TB + t.cB * dS * dS + c2s2 * dA * dA - kG * fma(t.sB, t.cAB, t.cB * t.sAB);
        gA[2] = 2.0 * t.sB * fma(t.cB, dA, dS);
        gA[3] = 2.0 * t.sB * dS;
        gA[4] = 1.0;
        gA[5] = -t.E;
        const double Q = fma(t.F * dA, dA, t.E * dB * fma(2.0, dA, dB));   // F dA^2 + E dB^2 + 2 E dA dB
        const double P = dA * fma(2.0, dA, 2.0 * dB) + dB * dB;            // 2 dA^2 + dB^2 + 2 dA dB
        gB[0] = kG * fma(-(2.0 + t.cB), t.sAB, 2.0 * t.E * t.sA);
        gB[1] = fma(-t.sB, TA, 2.0 * t.sB * TB) + fma(t.cB, Q, -t.sB * t.sB * P) +
                kG * (fma(-t.sB, t.cAB, -(2.0 + t.cB) * t.sAB) + 2.0 * t.sB * t.cA);
        gB[2] = 2.0 * t.sB * fma(t.F, dA, t.E * dB);
        gB[3] = 2.0 * t.E * t.sB * dS;
        gB[4] = t.E;
        gB[5] = -t.F;
    }
    // acceleration and d acc/dq [2x2], d acc/dqd [2x2], d acc/du [2x2] (row-major): quotient rule, D' = -2 cB sB
    MMPC_HD static void eval_acc_jac(const double* x, const double* u, double* acc, double* Fq, double* Fqd, double* Fu) {
        Terms t;
        terms(x, u, t);
        double gA[6], gB[6];
        grads(x, u, t, gA, gB);
        const double aA = -t.nA * t.iD, aB = t.nB * t.iD;
        acc[0] = aA;
        acc[1] = aB;
        const double rD = -2.0 * t.cB * t.sB * t.iD;   // D'/D
        // d(-nA/D) = -(gA - nA D'/D e_qB)/D ;  d(nB/D) = (gB - nB D'/D e_qB)/D
        Fq[0] = -gA[0] * t.iD;
        Fq[1] = fma(-gA[1], t.iD, -aA * rD);
        Fq[2] = gB[0] * t.iD;
        Fq[3] = fma(gB[1], t.iD, -aB * rD);
        Fqd[0] = -gA[2] * t.iD;
        Fqd[1] = -gA[3] * t.iD;
        Fqd[2] = gB[2] * t.iD;
        Fqd[3] = gB[3] * t.iD;
        Fu[0] = -gA[4] * t.iD;
        Fu[1] = -gA[5] * t.iD;
        Fu[2] = gB[4] * t.iD;
        Fu[3] = gB[5] * t.iD;
    }
    // W = lam[0] d^2 qA_ddot + lam[1] d^2 qB_ddot (6x6 row-major) = d^2 (psi / D), psi = -lam0 nA + lam1 nB:
    //   W_ij = psi_ij / D - (psi_i D_j + D_i psi_j) / D^2 + psi (2 D_i D_j / D^3 - D_ij / D^2),  D_i = D' [i == qB]
    MMPC_HD static void eval_hess(const double* x, const double* u, const double* lam, double* W) {
        Terms t;
        terms(x, u, t);
        double gA[6], gB[6];
        grads(x, u, t, gA, gB);
        const double dA = x[2], dB = x[3], TA = u[0], TB = u[1], dS = dA + dB;
        const double l0 = -lam[0], l1 = lam[1];   // psi = l0 nA + l1 nB
        const double c2s2 = fma(t.cB, t.cB, -t.sB * t.sB);
        const double Q = fma(t.F * dA, dA, t.E * dB * fma(2.0, dA, dB));
        const double P = dA * fma(2.0, dA, 2.0 * dB) + dB * dB;
        // second derivatives of nA, nB (nonzero pairs; T enters linearly, qA only through the gravity terms)
        const double A00 = kG * fma(-t.cB, t.cAB, 2.0 * t.cA);
        const double A01 = kG * fma(t.sB, t.sAB, -t.cB * t.cAB);
        const double A11 = t.cB * TB - t.sB * dS * dS - 4.0 * t.cB * t.sB * dA * dA -
                           2.0 * kG * fma(t.cB, t.cAB, -t.sB * t.sAB);
        const double A12 = 2.0 * fma(t.cB, dS, c2s2 * dA), A13 = 2.0 * t.cB * dS, A15 = t.sB;
        const double A22 = 2.0 * t.sB * t.E, A23 = 2.0 * t.sB, A33 = 2.0 * t.sB;
        const double B00 = kG * fma(-(2.0 + t.cB), t.cAB, 2.0 * t.E * t.cA);
        const double B01 = kG * (fma(t.sB, t.sAB, -(2.0 + t.cB) * t.cAB) - 2.0 * t.sB * t.sA);
        const double B11 = fma(-t.cB, TA, 2.0 * t.cB * TB) - t.sB * fma(3.0 * t.cB, P, Q) +
                           2.0 * kG * (fma(-t.E, t.cAB, t.sB * t.sAB) + t.cB * t.cA);
        const double B12 = fma(t.cB, 2.0 * fma(t.F, dA, t.E * dB), -t.sB * t.sB * (4.0 * dA + 2.0 * dB));
        const double B13 = 2.0 * dS * fma(t.E, t.cB, -t.sB * t.sB), B14 = -t.sB, B15 = 2.0 * t.sB;
        const double B22 = 2.0 * t.F * t.sB, B23 = 2.0 * t.E * t.sB, B33 = 2.0 * t.E * t.sB;
        double H[6][6];
#pragma unroll
        for (int i = 0; i < 6; ++i)
#pragma unroll
            for (int j = 0; j < 6; ++j) H[i][j] = 0.0;
        H[0][0] = fma(l0, A00, l1 * B00);
        H[0][1] = fma(l0, A01, l1 * B01);
        H[1][1] = fma(l0, A11, l1 * B11);
        H[1][2] = fma(l0, A12, l1 * B12);
        H[1][3] = fma(l0, A13, l1 * B13);
        H[1][4] = l1 * B14;
        H[1][5] = fma(l0, A15, l1 * B15);
        H[2][2] = fma(l0, A22, l1 * B22);
        H[2][3] = fma(l0, A23, l1 * B23);
        H[3][3] = fma(l0, A33, l1 * B33);
        double gp[6];
#pragma unroll
        for (int j = 0; j < 6; ++j) gp[j] = fma(l0, gA[j], l1 * gB[j]);
        const double psi = fma(l0, t.nA, l1 * t.nB);
        const double Dp = -2.0 * t.cB * t.sB, Dpp = -2.0 * c2s2;   // D', D'' (qB only)
        const double iD = t.iD, iD2 = iD * iD;
#pragma unroll
        for (int i = 0; i < 6; ++i)
#pragma unroll
            for (int j = i; j < 6; ++j) {
                double v = H[i][j] * iD;
                if (j == 1) v = fma(-gp[i] * Dp, iD2, v);   // -(psi_i D_j)/D^2
                if (i == 1) v = fma(-gp[j] * Dp, iD2, v);   // -(D_i psi_j)/D^2
                if (i == 1 && j == 1) v = fma(psi, fma(2.0 * Dp * Dp, iD, -Dpp) * iD2, v);
                W[i * 6 + j] = v;
                W[j * 6 + i] = v;
            }
    }
};

}  // namespace mmpc
