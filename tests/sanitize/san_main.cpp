// Host-code sanitizer driver (AddressSanitizer + UndefinedBehaviorSanitizer, no recovery):
// exercises the C oracle (oracle/reacher_ref.c: Philox resets, the fused distillation step
// on two OpenMP threads for both losses and both actors, ragged n, TF1 Adam) and the product's
// host-only C++ (csrc/gym_seed.cpp: sha512 -> MT19937 gym reset draws).  Built and run by
// tests/test_sanitizers.py; exits 0 and prints "san ok" when nothing was reported.
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <vector>

extern "C" {
int rdo_param_count(void);
void rdo_philox_reset(int64_t n, int64_t env_base, uint64_t seed, uint32_t episode, float* state);
void rdo_distill_step(int64_t n, int64_t n_global, int64_t env_base, uint64_t seed, int64_t step, float* state,
                      const float* tp, const float* tmu, const float* tsd, const float* sp, const float* smu,
                      const float* ssd, int loss, int act_student, int stagger, float* grad, double* metrics,
                      int nthreads);
void rdo_adam_tf1(int64_t n, float* theta, float* m, float* v, const float* g, float b1p, float b2p, float lr,
                  float b1, float b2, float eps);
int rd_gym_reset_draws(uint64_t seed, int32_t n_episodes, double* out);
}

int main() {
    const int P = rdo_param_count();
    std::vector<float> tp(P), sp(P), mu(11, 0.0f), sd(11, 1.0f), grad(P), m(P, 0.0f), v(P, 0.0f);
    uint32_t x = 12345u;
    auto rnd = [&] { x = x * 1664525u + 1013904223u; return ((x >> 8) * (1.0f / 16777216.0f) - 0.5f) * 0.2f; };
    for (int i = 0; i < P; ++i) { tp[i] = rnd(); sp[i] = rnd(); }
    tp[P - 2] = tp[P - 1] = -1.0f;   // logstd
    sp[P - 2] = sp[P - 1] = -0.5f;
    double checksum = 0.0;
    for (int64_t n : {1, 17, 257}) {
        std::vector<float> state(8 * n);
        rdo_philox_reset(n, 3, 7, 0, state.data());
        for (int loss = 0; loss < 2; ++loss)
            for (int act = 0; act < 2; ++act)
                for (int step = 0; step < 3; ++step) {
                    double met[4] = {0, 0, 0, 0};
                    rdo_distill_step(n, n, 3, 7, step, state.data(), tp.data(), mu.data(), sd.data(), sp.data(),
                                     mu.data(), sd.data(), loss, act, 1, grad.data(), met, 2);
                    rdo_adam_tf1(P, sp.data(), m.data(), v.data(), grad.data(), 0.9f, 0.999f, 1e-4f, 0.9f, 0.999f,
                                 1e-8f);
                    checksum += met[0] + met[1];
                }
    }
    std::vector<double> draws(6 * 25);
    if (rd_gym_reset_draws(0, 25, draws.data()) != 0) return 2;
    if (rd_gym_reset_draws(0, -1, draws.data()) == 0) return 3;   // bad argument reported
    for (double d : draws) checksum += d;
    std::printf("san ok %.6g\n", checksum);
    return 0;
}
