// Host-side equivalence check of stream.hip's var_land (the framing DP's variable-message
// landing) against parse_var, the full restatement the walk and the emit use: for random and
// well-formed byte windows, both wire formats, every position and several buffer ends,
// var_land(p) == (parse_var(limit = c0 + kC + kE - 1) == kOk && p + len < kC + kE ? p + len : 0xFF).
//   hipcc -O2 -std=c++17 -I minpaxos_amd/csrc tools/check/var_land_check.cpp -o /tmp/vlc && /tmp/vlc
// (host code only: no GPU call)
#include "../../minpaxos_amd/csrc/stream.hip"
#include <cstdio>
#include <random>
#include <vector>

using namespace mpx;

static uint32_t want(const std::vector<uint8_t>& b, uint64_t len, uint64_t c0, uint32_t p, int proto) {
    const Bytes by{b.data(), nullptr, 0, 0};
    const VarRes r = parse_var(by, len, c0 + kC + kE - 1, c0 + p, proto);
    const uint32_t q = p + r.f.len;
    return r.st == kOk && q < (uint32_t)(kC + kE) ? q : 0xFFu;
}

int main() {
    std::mt19937_64 rng(12345);
    uint64_t checked = 0, landed = 0;
    for (int it = 0; it < 400000; ++it) {
        std::vector<uint8_t> b(kC + kE + 64);
        const int mode = it % 4;
        for (auto& x : b) {
            const uint64_t r = rng();
            // mode 0: uniform bytes; 1: small bytes (short varints, small counts); 2: mostly
            // zero (n = m = 0 frames); 3: var codes and small values mixed
            x = mode == 0 ? (uint8_t)r : mode == 1 ? (uint8_t)(r % 8) : mode == 2 ? (uint8_t)(r % 16 == 0 ? r >> 8 : 0)
                                                 : (uint8_t)((r & 3) == 0 ? 9 + (r >> 8) % 4 : (r >> 16) % 6);
        }
        const uint64_t c0 = 0;
        const uint64_t lens[3] = {b.size(), (uint64_t)(rng() % b.size()), kC + kE - 1 + rng() % 3};
        for (uint64_t len : lens) {
            if (len > b.size()) len = b.size();
            const uint32_t e = (uint32_t)std::min(len - c0, (uint64_t)(kC + kE - 1));
            for (int proto : {MPX_MODE_MIN, MPX_MODE_CLASSIC}) {
                for (uint32_t p = 0; p < (uint32_t)kC && c0 + p < len; ++p) {
                    const uint32_t code = b[p];
                    if (flen(code, proto)) continue;
                    const uint32_t g = var_land(TileBytes{nullptr, nullptr, b.data()}, p, e, proto);
                    const uint32_t w = want(b, len, c0, p, proto);
                    ++checked;
                    landed += w != 0xFFu;
                    if (g != w) {
                        std::printf("MISMATCH it %d proto %d len %llu p %u: var_land %u parse_var %u\n", it,
                                    proto, (unsigned long long)len, p, g, w);
                        return 1;
                    }
                }
            }
        }
    }
    std::printf("var_land == parse_var on %llu variable-message positions (%llu landings)\n",
                (unsigned long long)checked, (unsigned long long)landed);
    return 0;
}
