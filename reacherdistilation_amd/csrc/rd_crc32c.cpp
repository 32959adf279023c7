// CRC32C (Castagnoli) on the host for the TF checkpoint reader / writer (tf_checkpoint.py):
// the masked CRC of every table block and the crc32c of every tensor's bytes.  Slicing-by-8
// (eight 256-entry tables, one 8-byte word per step) everywhere, and the SSE4.2 crc32
// instruction (which computes exactly this polynomial) where the host CPU has it; the per-byte
// Python loop it replaces ran at ~2 MB/s.  Reflected polynomial 0x82F63B78,
// init/final xor ~0: check value crc32c("123456789") = 0xE3069283.
#include <stdint.h>
#include <string.h>

#include "../../include/reacher.h"

namespace {

struct Tables {
    uint32_t t[8][256];
    Tables() {
        for (uint32_t i = 0; i < 256; ++i) {
            uint32_t c = i;
            for (int k = 0; k < 8; ++k) c = (c & 1u) ? (c >> 1) ^ 0x82F63B78u : c >> 1;
            t[0][i] = c;
        }
        for (uint32_t i = 0; i < 256; ++i)
            for (int s = 1; s < 8; ++s) t[s][i] = (t[s - 1][i] >> 8) ^ t[0][t[s - 1][i] & 0xFFu];
    }
};

const Tables& tables() {
    static const Tables tb;
    return tb;
}

// c is the running (pre-inverted) register on entry and exit
__attribute__((target("sse4.2"))) uint32_t crc_hw(const uint8_t* data, int64_t n, uint32_t c) {
    uint64_t c64 = c;
    int64_t i = 0;
    for (; i + 8 <= n; i += 8) {
        uint64_t w;
        memcpy(&w, data + i, 8);
        c64 = __builtin_ia32_crc32di(c64, w);
    }
    uint32_t c32 = (uint32_t)c64;
    for (; i < n; ++i) c32 = __builtin_ia32_crc32qi(c32, data[i]);
    return c32;
}

bool have_hw() {
    static const bool hw = __builtin_cpu_supports("sse4.2");
    return hw;
}

}  // namespace

extern "C" uint32_t rd_crc32c(const uint8_t* data, int64_t n, uint32_t crc) {
    uint32_t c = ~crc;
    if (!data || n <= 0) return ~c;
    if (have_hw()) return ~crc_hw(data, n, c);
    const Tables& tb = tables();
    int64_t i = 0;
    for (; i + 8 <= n; i += 8) {   // little-endian host (x86-64)
        uint32_t lo, hi;
        memcpy(&lo, data + i, 4);
        memcpy(&hi, data + i + 4, 4);
        lo ^= c;
        c = tb.t[7][lo & 0xFFu] ^ tb.t[6][(lo >> 8) & 0xFFu] ^ tb.t[5][(lo >> 16) & 0xFFu] ^ tb.t[4][lo >> 24] ^
            tb.t[3][hi & 0xFFu] ^ tb.t[2][(hi >> 8) & 0xFFu] ^ tb.t[1][(hi >> 16) & 0xFFu] ^ tb.t[0][hi >> 24];
    }
    for (; i < n; ++i) c = tb.t[0][(c ^ data[i]) & 0xFFu] ^ (c >> 8);
    return ~c;
}
