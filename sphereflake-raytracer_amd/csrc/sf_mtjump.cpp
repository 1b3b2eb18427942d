// sf_mtjump.cpp -- jump-ahead for std::mt19937 (host side of the parallel frame-less draws).
//
// The reference worker draws its packet scrambles from std::mt19937 (Sphereflake.cpp:88-90, 139-141); the
// device reproduces that stream bit for bit. One sequential generator bounds a 2^18-packet batch (524 288
// draws), so the batch is cut into K contiguous segments generated in parallel, each starting from the state
// the stream has at its first draw.
//
// MT19937 is linear over GF(2): with W_n = (x_n, ..., x_{n+623}) the window of raw (untempered) words,
// W_{n+1} = A W_n, and A's characteristic polynomial phi (degree 19937, primitive) gives
//     W_{n+J} = sum_i a_i W_{n+i},    sum_i a_i t^i = t^J mod phi,
// i.e. word w of the jumped window is the XOR of x_{n+i+w} over the set coefficients i -- a convolution of
// the raw sequence with the jump polynomial, which the device evaluates (sf_mt_jump_partial). Here: phi by
// Berlekamp-Massey on one bit of the generator's output (phi is irreducible, so any nonzero bit sequence of
// the generator has exactly phi as its minimal polynomial), and t^J mod phi by square-and-multiply.
// Polynomials are little-endian uint64 bit arrays.
#include <cstdint>
#include <cstring>
#include <map>
#include <mutex>
#include <random>
#include <vector>

#include "sf_internal.h"

namespace sfhost {
namespace {

constexpr int kDeg = 19937;
constexpr int kWords = (kDeg + 64) / 64;   // degree <= 19937 fits (313 words)

using Poly = std::vector<uint64_t>;

inline int get_bit(const Poly& p, int i) { return (int)((p[(size_t)i >> 6] >> (i & 63)) & 1u); }
inline void flip_bit(Poly& p, int i) { p[(size_t)i >> 6] ^= 1ull << (i & 63); }

// a ^= b << s (bit shift), a sized to hold the result
void xor_shifted(Poly& a, const Poly& b, int s, int nbits_b)
{
    const int ws = s >> 6, bs = s & 63;
    const int nb = (nbits_b + 63) >> 6;
    for (int k = 0; k < nb; ++k) {
        const uint64_t v = b[(size_t)k];
        if (!v) continue;
        a[(size_t)(k + ws)] ^= v << bs;
        if (bs && (size_t)(k + ws + 1) < a.size()) a[(size_t)(k + ws + 1)] ^= v >> (64 - bs);
    }
}

// Berlekamp-Massey over GF(2): the connection polynomial C (C_0 = 1) of the shortest LFSR generating s.
Poly berlekamp_massey(const std::vector<uint8_t>& s, int& L)
{
    const int n = (int)s.size();
    const size_t W = (size_t)(n + 64) / 64 + 2;
    Poly C(W, 0), B(W, 0), T;
    C[0] = B[0] = 1;
    L = 0;
    int m = 1;
    // the sequence reversed as a bit array: rs[j] = s[n - 1 - j]; the discrepancy
    // d = s_N ^ sum_{i=1..L} C_i s_{N-i} = parity of C & (rs shifted to start at bit n - 1 - N), word by word
    Poly rs(W + 1, 0);
    for (int j = 0; j < n; ++j)
        if (s[(size_t)(n - 1 - j)]) flip_bit(rs, j);
    auto rs_word = [&](int bit) -> uint64_t {   // 64 bits of rs from `bit`
        const size_t q = (size_t)bit >> 6;
        const int r = bit & 63;
        const uint64_t lo = rs[q], hi = q + 1 < rs.size() ? rs[q + 1] : 0ull;
        return r ? (lo >> r) | (hi << (64 - r)) : lo;
    };
    for (int N = 0; N < n; ++N) {
        const int base = n - 1 - N;   // rs bit of s_N
        uint64_t acc = 0;
        for (int q = 0; q <= L / 64; ++q) {   // C bits 64 q .. 64 q + 63 against s_{N - 64 q}, ...
            uint64_t c = C[(size_t)q];
            if (q == 0) c &= ~1ull;                                     // (C_0 is not part of the sum)
            if (64 * q + 63 > L) c &= (L - 64 * q >= 63) ? ~0ull : ((2ull << (L - 64 * q)) - 1ull);
            acc ^= c & rs_word(base + 64 * q);
        }
        const int d = (s[(size_t)N] ^ __builtin_parityll(acc)) & 1;
        if (!d) {
            ++m;
        } else if (2 * L <= N) {
            T = C;
            xor_shifted(C, B, m, n + 1);
            L = N + 1 - L;
            B = T;
            m = 1;
        } else {
            xor_shifted(C, B, m, n + 1);
            ++m;
        }
    }
    return C;
}

// phi(t) = t^L C(1/t): coefficient of t^k is C_{L-k}
const Poly& charpoly()
{
    static Poly phi;
    static std::once_flag once;
    std::call_once(once, [] {
        std::mt19937 g(5489u);
        std::vector<uint8_t> s(2 * kDeg + 64);
        for (auto& b : s) b = (uint8_t)(g() & 1u);
        int L = 0;
        const Poly C = berlekamp_massey(s, L);
        phi.assign(kWords, 0);
        for (int k = 0; k <= L; ++k)
            if (get_bit(C, L - k)) flip_bit(phi, k);
        // L == kDeg for MT19937 (checked by the tests through sf_mt19937_jump against the generator)
    });
    return phi;
}

// r (degree < 2 kDeg) mod phi, in place; r sized 2 * kWords
void reduce(Poly& r)
{
    const Poly& phi = charpoly();
    for (int d = 2 * kDeg - 2; d >= kDeg; --d)
        if (get_bit(r, d)) xor_shifted(r, phi, d - kDeg, kDeg + 1);
    r.resize(kWords);
    // clear bits >= kDeg of the last word
    r[kWords - 1] &= (1ull << (kDeg & 63)) - 1ull;
}

Poly mulmod(const Poly& a, const Poly& b)
{
    Poly r(2 * kWords, 0);
    for (int i = 0; i < kDeg; ++i)
        if (get_bit(a, i)) xor_shifted(r, b, i, kDeg);
    reduce(r);
    return r;
}

Poly sqrmod(const Poly& a)
{
    Poly r(2 * kWords, 0);
    for (int i = 0; i < kDeg; ++i)
        if (get_bit(a, i)) flip_bit(r, 2 * i);
    reduce(r);
    return r;
}

// t * a mod phi
Poly mulx(const Poly& a)
{
    Poly r(2 * kWords, 0);
    xor_shifted(r, a, 1, kDeg);
    reduce(r);
    return r;
}

Poly xpow(uint64_t J)   // t^J mod phi
{
    Poly r(kWords, 0);
    r[0] = 1;
    if (J == 0) return r;
    int top = 63;
    while (!((J >> top) & 1u)) --top;
    for (int b = top; b >= 0; --b) {
        r = sqrmod(r);
        if ((J >> b) & 1u) r = mulx(r);
    }
    return r;
}

}  // namespace

int mt_poly_words() { return kWords; }

// t^(j L) mod phi for j = 0 .. K - 1, K x kWords words (cached per (L, K))
const uint64_t* mt_jump_polys(uint64_t L, uint32_t K)
{
    static std::mutex mu;
    static std::map<std::pair<uint64_t, uint32_t>, Poly> cache;
    std::lock_guard<std::mutex> lk(mu);
    auto it = cache.find({ L, K });
    if (it != cache.end()) return it->second.data();
    Poly all((size_t)K * kWords, 0);
    Poly cur(kWords, 0);
    cur[0] = 1;
    const Poly step = xpow(L);
    for (uint32_t j = 0; j < K; ++j) {
        std::memcpy(&all[(size_t)j * kWords], cur.data(), kWords * 8);
        if (j + 1 < K) cur = mulmod(cur, step);
    }
    return cache.emplace(std::make_pair(L, K), std::move(all)).first->second.data();
}

// Host reference: the std::mt19937 state (624 words + next index, libstdc++ layout) after `outputs` more
// draws, by the polynomial jump (tests compare it with the generator stepped one draw at a time).
// With the buffer holding raw words x_0..x_623 and next index p, the draws still in the buffer are
// temper(x_p..x_623); after those the sequence continues with x_624, x_625, ..., and the buffer itself is the
// window V_0 = (x_0..x_623) that x_624 is twisted from. m draws past the buffer leave the window V_m =
// (x_m..x_{m+623}) = (t^m mod phi)(A) V_0, whose word k is the XOR of x_{i+k} over the polynomial's set
// coefficients i; as a std::mt19937 state that is the buffer V_m with next index 624.
void mt_jump(const uint32_t in[625], uint64_t outputs, uint32_t out[625])
{
    const uint32_t pos = in[624] > 624u ? 624u : in[624];
    if (outputs <= 624u - pos) {   // still inside the buffer
        std::memcpy(out, in, 624 * 4);
        out[624] = pos + (uint32_t)outputs;
        return;
    }
    const uint64_t m = outputs - (624u - pos);   // draws past the buffer
    std::vector<uint32_t> x((size_t)kDeg + 624 + 624);
    std::memcpy(x.data(), in, 624 * 4);
    for (size_t k = 624; k < x.size(); ++k) {
        const uint32_t y = (x[k - 624] & 0x80000000u) | (x[k - 623] & 0x7fffffffu);
        x[k] = x[k - 227] ^ (y >> 1) ^ ((y & 1u) ? 0x9908b0dfu : 0u);
    }
    const Poly a = xpow(m);
    uint32_t w[624] = {};
    for (int i = 0; i < kDeg; ++i)
        if (get_bit(a, i))
            for (int k = 0; k < 624; ++k) w[k] ^= x[(size_t)i + k];
    std::memcpy(out, w, sizeof w);
    out[624] = 624u;
}

}  // namespace sfhost
