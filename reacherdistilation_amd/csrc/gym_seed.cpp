// Host-side gym seeding for Reacher-v2 resets (native, no Python on the path).
//
// Reference: make_mujoco_env("Reacher-v2", 0) (reference mlp_train.py:21) ends in
// env.seed(0) -> gym/utils/seeding.py np_random(seed):
//     rng = RandomState(); rng.seed(_int_list_from_bigint(hash_seed(create_seed(seed))))
//   hash_seed: sha512(str(seed).encode()).digest()[:8] -> little-endian uint32 words
//   RandomState.seed(list) = MT19937 init_by_array; uniform = low + (high-low)*res53()
// and every env.reset() runs ReacherEnv.reset_model:
//     qpos = U(-.1,.1, 4); goal = U(-.2,.2, 2) until |goal| < 2; qvel = U(-.005,.005, 4)
// (gym 0.10.5, requirement.txt:20).  Verified bit-exact against the reference fixture's
// 25 resets (tests/test_env_host.py).
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <string>
#include <vector>

#include "../../include/reacher.h"

namespace {

// ---------------------------------------------------------------- SHA-512 (FIPS 180-4)
const uint64_t K512[80] = {
    0x428a2f98d728ae22ULL, 0x7137449123ef65cdULL, 0xb5c0fbcfec4d3b2fULL, 0xe9b5dba58189dbbcULL,
    0x3956c25bf348b538ULL, 0x59f111f1b605d019ULL, 0x923f82a4af194f9bULL, 0xab1c5ed5da6d8118ULL,
    0xd807aa98a3030242ULL, 0x12835b0145706fbeULL, 0x243185be4ee4b28cULL, 0x550c7dc3d5ffb4e2ULL,
    0x72be5d74f27b896fULL, 0x80deb1fe3b1696b1ULL, 0x9bdc06a725c71235ULL, 0xc19bf174cf692694ULL,
    0xe49b69c19ef14ad2ULL, 0xefbe4786384f25e3ULL, 0x0fc19dc68b8cd5b5ULL, 0x240ca1cc77ac9c65ULL,
    0x2de92c6f592b0275ULL, 0x4a7484aa6ea6e483ULL, 0x5cb0a9dcbd41fbd4ULL, 0x76f988da831153b5ULL,
    0x983e5152ee66dfabULL, 0xa831c66d2db43210ULL, 0xb00327c898fb213fULL, 0xbf597fc7beef0ee4ULL,
    0xc6e00bf33da88fc2ULL, 0xd5a79147930aa725ULL, 0x06ca6351e003826fULL, 0x142929670a0e6e70ULL,
    0x27b70a8546d22ffcULL, 0x2e1b21385c26c926ULL, 0x4d2c6dfc5ac42aedULL, 0x53380d139d95b3dfULL,
    0x650a73548baf63deULL, 0x766a0abb3c77b2a8ULL, 0x81c2c92e47edaee6ULL, 0x92722c851482353bULL,
    0xa2bfe8a14cf10364ULL, 0xa81a664bbc423001ULL, 0xc24b8b70d0f89791ULL, 0xc76c51a30654be30ULL,
    0xd192e819d6ef5218ULL, 0xd69906245565a910ULL, 0xf40e35855771202aULL, 0x106aa07032bbd1b8ULL,
    0x19a4c116b8d2d0c8ULL, 0x1e376c085141ab53ULL, 0x2748774cdf8eeb99ULL, 0x34b0bcb5e19b48a8ULL,
    0x391c0cb3c5c95a63ULL, 0x4ed8aa4ae3418acbULL, 0x5b9cca4f7763e373ULL, 0x682e6ff3d6b2b8a3ULL,
    0x748f82ee5defb2fcULL, 0x78a5636f43172f60ULL, 0x84c87814a1f0ab72ULL, 0x8cc702081a6439ecULL,
    0x90befffa23631e28ULL, 0xa4506cebde82bde9ULL, 0xbef9a3f7b2c67915ULL, 0xc67178f2e372532bULL,
    0xca273eceea26619cULL, 0xd186b8c721c0c207ULL, 0xeada7dd6cde0eb1eULL, 0xf57d4f7fee6ed178ULL,
    0x06f067aa72176fbaULL, 0x0a637dc5a2c898a6ULL, 0x113f9804bef90daeULL, 0x1b710b35131c471bULL,
    0x28db77f523047d84ULL, 0x32caab7b40c72493ULL, 0x3c9ebe0a15c9bebcULL, 0x431d67c49c100d4cULL,
    0x4cc5d4becb3e42b6ULL, 0x597f299cfc657e2aULL, 0x5fcb6fab3ad6faecULL, 0x6c44198c4a475817ULL};

inline uint64_t rotr(uint64_t x, int n) { return (x >> n) | (x << (64 - n)); }

void sha512(const uint8_t* msg, size_t len, uint8_t out[64]) {
    uint64_t H[8] = {0x6a09e667f3bcc908ULL, 0xbb67ae8584caa73bULL, 0x3c6ef372fe94f82bULL,
                     0xa54ff53a5f1d36f1ULL, 0x510e527fade682d1ULL, 0x9b05688c2b3e6c1fULL,
                     0x1f83d9abfb41bd6bULL, 0x5be0cd19137e2179ULL};
    std::vector<uint8_t> m(msg, msg + len);
    m.push_back(0x80);
    while (m.size() % 128 != 112) m.push_back(0);
    for (int i = 0; i < 8; ++i) m.push_back(0);                       // high 64 bits of length
    const uint64_t bits = (uint64_t)len * 8;
    for (int i = 7; i >= 0; --i) m.push_back((uint8_t)(bits >> (8 * i)));
    for (size_t blk = 0; blk < m.size(); blk += 128) {
        uint64_t W[80];
        for (int t = 0; t < 16; ++t) {
            uint64_t w = 0;
            for (int b = 0; b < 8; ++b) w = (w << 8) | m[blk + 8 * t + b];
            W[t] = w;
        }
        for (int t = 16; t < 80; ++t) {
            const uint64_t s0 = rotr(W[t - 15], 1) ^ rotr(W[t - 15], 8) ^ (W[t - 15] >> 7);
            const uint64_t s1 = rotr(W[t - 2], 19) ^ rotr(W[t - 2], 61) ^ (W[t - 2] >> 6);
            W[t] = W[t - 16] + s0 + W[t - 7] + s1;
        }
        uint64_t a = H[0], b = H[1], c = H[2], d = H[3], e = H[4], f = H[5], g = H[6], h = H[7];
        for (int t = 0; t < 80; ++t) {
            const uint64_t S1 = rotr(e, 14) ^ rotr(e, 18) ^ rotr(e, 41);
            const uint64_t ch = (e & f) ^ (~e & g);
            const uint64_t t1 = h + S1 + ch + K512[t] + W[t];
            const uint64_t S0 = rotr(a, 28) ^ rotr(a, 34) ^ rotr(a, 39);
            const uint64_t mj = (a & b) ^ (a & c) ^ (b & c);
            const uint64_t t2 = S0 + mj;
            h = g; g = f; f = e; e = d + t1; d = c; c = b; b = a; a = t1 + t2;
        }
        H[0] += a; H[1] += b; H[2] += c; H[3] += d; H[4] += e; H[5] += f; H[6] += g; H[7] += h;
    }
    for (int i = 0; i < 8; ++i)
        for (int b = 0; b < 8; ++b) out[8 * i + b] = (uint8_t)(H[i] >> (56 - 8 * b));
}

// ---------------------------------------------------------------- MT19937 (numpy legacy)
struct MT {
    uint32_t s[624];
    int i = 625;
    void init_genrand(uint32_t seed) {
        s[0] = seed;
        for (i = 1; i < 624; ++i) s[i] = 1812433253u * (s[i - 1] ^ (s[i - 1] >> 30)) + (uint32_t)i;
    }
    void init_by_array(const uint32_t* key, int n) {
        init_genrand(19650218u);
        int a = 1, b = 0;
        for (int k = (624 > n ? 624 : n); k; --k) {
            s[a] = (s[a] ^ ((s[a - 1] ^ (s[a - 1] >> 30)) * 1664525u)) + key[b] + (uint32_t)b;
            ++a; ++b;
            if (a >= 624) { s[0] = s[623]; a = 1; }
            if (b >= n) b = 0;
        }
        for (int k = 623; k; --k) {
            s[a] = (s[a] ^ ((s[a - 1] ^ (s[a - 1] >> 30)) * 1566083941u)) - (uint32_t)a;
            ++a;
            if (a >= 624) { s[0] = s[623]; a = 1; }
        }
        s[0] = 0x80000000u;
        i = 624;
    }
    uint32_t next() {
        if (i >= 624) {
            for (int k = 0; k < 624; ++k) {
                const uint32_t y = (s[k] & 0x80000000u) | (s[(k + 1) % 624] & 0x7fffffffu);
                s[k] = s[(k + 397) % 624] ^ (y >> 1) ^ ((y & 1u) ? 0x9908b0dfu : 0u);
            }
            i = 0;
        }
        uint32_t y = s[i++];
        y ^= y >> 11;
        y ^= (y << 7) & 0x9d2c5680u;
        y ^= (y << 15) & 0xefc60000u;
        y ^= y >> 18;
        return y;
    }
    double res53() {
        const uint32_t a = next() >> 5, b = next() >> 6;
        return (a * 67108864.0 + b) / 9007199254740992.0;
    }
    double uniform(double lo, double hi) { return lo + (hi - lo) * res53(); }
};

}  // namespace

extern "C" int rd_gym_reset_draws(uint64_t seed, int32_t n_episodes, double* out) {
    if (!out || n_episodes < 0) return RD_EINVAL;
    // create_seed(int): a % 2**64; hash_seed: sha512(str(a))[:8]
    char buf[32];
    const int len = snprintf(buf, sizeof buf, "%llu", (unsigned long long)seed);
    uint8_t dig[64];
    sha512((const uint8_t*)buf, (size_t)len, dig);
    // _bigint_from_bytes pads 8 bytes to 12 -> 3 LE uint32 words; _int_list_from_bigint
    // drops the high zero words (and maps 0 -> [0]).
    uint32_t w[3] = {0, 0, 0};
    for (int k = 0; k < 2; ++k)
        w[k] = (uint32_t)dig[4 * k] | ((uint32_t)dig[4 * k + 1] << 8) |
               ((uint32_t)dig[4 * k + 2] << 16) | ((uint32_t)dig[4 * k + 3] << 24);
    int nw = w[1] ? 2 : 1;
    MT mt;
    mt.init_by_array(w, nw);
    for (int e = 0; e < n_episodes; ++e) {
        double qpos[4], goal[2], qvel[4];
        for (double& q : qpos) q = mt.uniform(-0.1, 0.1);
        for (;;) {
            goal[0] = mt.uniform(-0.2, 0.2);
            goal[1] = mt.uniform(-0.2, 0.2);
            if (std::sqrt(goal[0] * goal[0] + goal[1] * goal[1]) < 2.0) break;
        }
        for (double& v : qvel) v = mt.uniform(-0.005, 0.005);
        double* o = out + 6 * e;
        o[0] = qpos[0]; o[1] = qpos[1]; o[2] = qvel[0]; o[3] = qvel[1]; o[4] = goal[0]; o[5] = goal[1];
    }
    return RD_OK;
}
