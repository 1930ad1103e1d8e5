// Host builds of the built-in 2-link arm's device derivative code: the SX-generated Hessian
// (mahi-mpc_amd/csrc/two_link_hess_gen.h) and the hand-written closed form (mahi-mpc_amd/csrc/two_link_fast.h).
// TEST INFRASTRUCTURE ONLY (see mmpc_oracle.h): tests/test_sx_models.py compares both with the oracle's
// independent dual / hyper-dual restatement (oracle_two_link_jac, oracle_two_link_hess).
#include <math.h>

#define MMPC_HD
#include "two_link_hess_gen.h"
#include "two_link_fast.h"

extern "C" void builtin_two_link_hess(const double* x, const double* u, const double* lam_acc, double* W) {
    mmpc::TwoLinkArmHess::eval_hess(x, u, lam_acc, W);
}

extern "C" void fast_two_link_hess(const double* x, const double* u, const double* lam_acc, double* W) {
    mmpc::TwoLinkFast::eval_hess(x, u, lam_acc, W);
}

// xd[4] and the acceleration partials Fq, Fqd, Fu (2x2 row-major each)
extern "C" void fast_two_link_acc_jac(const double* x, const double* u, double* xd, double* Fq, double* Fqd,
                                      double* Fu) {
    mmpc::TwoLinkFast::eval(x, u, xd);
    double acc[2];
    mmpc::TwoLinkFast::eval_acc_jac(x, u, acc, Fq, Fqd, Fu);
}
