// Host-side AddressSanitizer check of the C ABI's descriptor validation
// (sanitizers on host code only -- GPU ASan is not
// available on this pool).  Built by `make -C calibration-normalizing-flows_amd/csrc
// asan` against libcnf_hip_asan.so (cnf_abi.hip's host code instrumented) and
// run by tests/test_asan.py in the build container, no GPU needed: every
// call below either validates and returns, or sizes plans on the host.
//
// Seeded random descriptors -- valid, out of range, malformed hidden widths,
// random_flip permutation tables with out-of-range / duplicate entries,
// unknown option bits -- each through every size query and every launching
// entry point with a rejected argument (negative batch, NULL blob), so ASan
// sees the validation code read exactly the caller's arrays: the permutation
// table is a heap block of exactly L*D int64s.
#include <algorithm>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <random>
#include <vector>

#include "cnf.h"

static int g_fail = 0;
#define EXPECT(c)                                                     \
  do {                                                                \
    if (!(c)) {                                                       \
      std::fprintf(stderr, "abi_check: %s failed (line %d)\n", #c, __LINE__); \
      ++g_fail;                                                       \
    }                                                                 \
  } while (0)

static bool is_status(int st) { return st <= 0 && st >= -6; }

int main(int argc, char** argv) {
  const int iters = argc > 1 ? std::atoi(argv[1]) : 3000;
  std::mt19937_64 rng(20261018);
  auto U = [&](int lo, int hi) { return (int)std::uniform_int_distribution<int>(lo, hi)(rng); };
  EXPECT(cnf_abi_version() == CNF_ABI_VERSION);
  for (int st = -8; st <= 1; ++st) EXPECT(cnf_strerror(st) != nullptr);
  int n_ok = 0;
  for (int it = 0; it < iters; ++it) {
    cnf_desc d;
    std::memset(&d, 0, sizeof d);
    d.abi_version = U(0, 19) == 0 ? U(-3, 5) : CNF_ABI_VERSION;
    d.dim = U(0, 9) == 0 ? U(-4, 300) : U(2, 128);
    d.n_layers = U(0, 19) == 0 ? U(-2, 0) : U(1, 14);
    d.n_hidden = U(0, 19) == 0 ? U(-1, CNF_MAX_HIDDEN + 2) : U(0, 3);
    for (int i = 0; i < CNF_MAX_HIDDEN; ++i)
      d.hidden[i] = U(0, 29) == 0 ? U(-2, 700) : U(1, 160);
    d.scale = U(0, 29) == 0 ? 2 : U(0, 1);
    d.shift = U(0, 29) == 0 ? -1 : U(0, 1);
    d.strict_nan = U(0, 3) == 0;
    d.options = U(0, 9) == 0 ? U(0, 31) : (U(0, 3) == 0 ? CNF_OPT_NO_SGPR : 0);
    std::vector<int64_t>* perms = nullptr;
    if (d.dim >= 2 && d.dim <= CNF_MAX_DIM && d.n_layers >= 1 && U(0, 2) == 0) {
      perms = new std::vector<int64_t>((size_t)d.n_layers * d.dim);
      for (int l = 0; l < d.n_layers; ++l) {
        int64_t* p = perms->data() + (size_t)l * d.dim;
        for (int j = 0; j < d.dim; ++j) p[j] = j;
        std::shuffle(p, p + d.dim, rng);
        const int kind = U(0, 9);
        if (kind == 0) p[0] = -1;                                   // no perm on this layer
        else if (kind == 1) p[U(0, d.dim - 1)] = d.dim + U(0, 5);  // out of range
        else if (kind == 2) p[U(0, d.dim - 1)] = p[(U(1, d.dim - 1))];  // duplicate (maybe)
      }
      d.perms = perms->data();
    }
    int64_t nf = -1;
    int32_t nt = -1;
    size_t bytes = 0, ws = 0;
    const int s0 = cnf_param_count(&d, &nf);
    EXPECT(is_status(s0));
    EXPECT(is_status(cnf_param_tensor_count(&d, &nt)));
    const int s1 = cnf_prepared_bytes(&d, &bytes);
    EXPECT(is_status(s1));
    EXPECT(cnf_kernel_name(&d) != nullptr);
    const int64_t B = U(0, 4) == 0 ? -U(1, 9) : (int64_t)U(0, 1 << 20);
    EXPECT(is_status(cnf_forward_loss_workspace_bytes(&d, B, &ws)));
    EXPECT(is_status(cnf_vjp_workspace_bytes(&d, B, &ws)));
    EXPECT(is_status(cnf_vjp_inverse_workspace_bytes(&d, B, &ws)));
    if (s0 == CNF_OK) {
      ++n_ok;
      // an empty stack (no s- and no t-net) has no parameters
      const bool nets = d.scale || d.shift;
      EXPECT(nets ? (nf > 0 && nt > 0) : (nf == 0 && nt == 0));
      EXPECT(s1 == CNF_OK && bytes > 0);
    }
    // launching entry points with a rejected argument: no launch may happen
    float dummy[4] = {0, 0, 0, 0};
    const int64_t nb = -1 - U(0, 3);
    EXPECT(cnf_forward(&d, nullptr, dummy, dummy, dummy, nullptr, nb, nullptr) < 0);
    EXPECT(cnf_inverse(&d, nullptr, dummy, dummy, dummy, nullptr, 4, nullptr) < 0);
    EXPECT(cnf_forward_loss(&d, nullptr, dummy, nullptr, CNF_LOSS_CAL, 1.f, nullptr, nullptr,
                            dummy, 4, nullptr, 0, nullptr) < 0);
    EXPECT(cnf_predict(&d, nullptr, dummy, dummy, dummy, nullptr, nb, nullptr) < 0);
    EXPECT(cnf_vjp(&d, nullptr, dummy, nullptr, nullptr, nullptr, dummy, nullptr, nb, nullptr, 0,
                   nullptr) < 0);
    EXPECT(cnf_loss_vjp(&d, nullptr, dummy, nullptr, 7, 1.f, 1.f, dummy, dummy, nullptr, 4,
                        nullptr, 0, nullptr) < 0);
    EXPECT(cnf_vjp_inverse(&d, nullptr, dummy, nullptr, nullptr, nullptr, dummy, nullptr, nb,
                           nullptr, 0, nullptr) < 0);
    // (an empty stack -- no s- or t-net -- has nothing to update: CNF_OK, no launch)
    EXPECT(cnf_adam_step(&d, nullptr, dummy, dummy, dummy, 1, 1e-3, 0.9, 0.999, 1e-8, 0.0,
                         nullptr) <= 0);
    EXPECT(cnf_guard_nonfinite(dummy, -1, nullptr, nullptr) < 0);
    delete perms;
  }
  EXPECT(cnf_param_count(nullptr, nullptr) == CNF_ERR_NULL);
  EXPECT(n_ok > iters / 10);
  std::printf("{\"iters\": %d, \"valid_descriptors\": %d, \"failures\": %d}\n", iters, n_ok, g_fail);
  return g_fail ? 1 : 0;
}
