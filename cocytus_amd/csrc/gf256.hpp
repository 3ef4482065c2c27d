// gf256.hpp -- GF(2^8) field arithmetic for libcocytus_ec (host + device, constexpr).
//
// Field of Jerasure 2.x / GF-Complete w = 8 (the library Cocytus links as
// -lJerasure, /root/reference/Makefile.am:46,49): primitive polynomial
// x^8 + x^4 + x^3 + x^2 + 1 (0x11D), generator 2.  Built at compile time; this
// is product code and shares nothing with oracle/.
#pragma once

#include <stdint.h>

namespace cec {

constexpr unsigned kPoly = 0x11D;

struct GfTables {
    uint8_t exp[512];   // exp[i] = 2^i, doubled so exp[log a + log b] needs no mod
    int16_t log[256];   // log[0] = -1
    constexpr GfTables() : exp(), log() {
        unsigned x = 1;
        for (int i = 0; i < 255; ++i) {
            exp[i] = static_cast<uint8_t>(x);
            exp[i + 255] = static_cast<uint8_t>(x);
            log[x] = static_cast<int16_t>(i);
            x <<= 1;
            if (x & 0x100u) x ^= kPoly;
        }
        exp[510] = exp[0];
        exp[511] = exp[1];
        log[0] = -1;
    }
};

inline constexpr GfTables kGf{};

constexpr int gf_mul(int a, int b) {
    a &= 0xFF;
    b &= 0xFF;
    return (a == 0 || b == 0) ? 0 : kGf.exp[kGf.log[a] + kGf.log[b]];
}

constexpr int gf_inv(int a) {  // a != 0
    return kGf.exp[(255 - kGf.log[a & 0xFF]) % 255];
}

constexpr int gf_div(int a, int b) {  // b != 0
    return (a & 0xFF) == 0 ? 0 : kGf.exp[kGf.log[a & 0xFF] + 255 - kGf.log[b & 0xFF]];
}

// Byte-permute product tables of one coefficient c (the PERM engine).
// Multiplication by c is GF(2)-linear in x, so with x = x[2:0] ^ x[5:3]<<3 ^ x[7:6]<<6:
//   c*x = T0[x & 7] ^ T1[(x >> 3) & 7] ^ T2[x >> 6]
// T0, T1 have 8 byte entries (two dwords each), T2 four (one dword).  One
// v_perm_b32 looks up 4 packed bytes in an 8-byte table, so a packed dword of 4
// bytes costs 3 perms per coefficient.  Layout: {T0[0..3], T0[4..7], T1[0..3],
// T1[4..7], T2[0..3]}, little-endian bytes.
struct PermTab {
    uint32_t w[5];
};

constexpr PermTab make_perm_tab(int c) {
    PermTab t{};
    for (int i = 0; i < 8; ++i) {
        t.w[i >> 2] |= static_cast<uint32_t>(gf_mul(c, i)) << (8 * (i & 3));
        t.w[2 + (i >> 2)] |= static_cast<uint32_t>(gf_mul(c, i << 3)) << (8 * (i & 3));
    }
    for (int i = 0; i < 4; ++i) t.w[4] |= static_cast<uint32_t>(gf_mul(c, i << 6)) << (8 * i);
    return t;
}

// Jerasure-compatible Gauss-Jordan inverse (row swaps, clobbers mat); -1 if singular.
inline int invert_matrix(int *mat, int *inv, int n) {
    for (int i = 0; i < n; ++i)
        for (int j = 0; j < n; ++j) inv[i * n + j] = (i == j);
    for (int i = 0; i < n; ++i) {
        if (mat[i * n + i] == 0) {
            int r = i + 1;
            while (r < n && mat[r * n + i] == 0) ++r;
            if (r == n) return -1;
            for (int c = 0; c < n; ++c) {
                int t = mat[i * n + c]; mat[i * n + c] = mat[r * n + c]; mat[r * n + c] = t;
                t = inv[i * n + c]; inv[i * n + c] = inv[r * n + c]; inv[r * n + c] = t;
            }
        }
        const int piv = mat[i * n + i];
        if (piv != 1) {
            const int s = gf_inv(piv);
            for (int c = 0; c < n; ++c) {
                mat[i * n + c] = gf_mul(mat[i * n + c], s);
                inv[i * n + c] = gf_mul(inv[i * n + c], s);
            }
        }
        for (int r = 0; r < n; ++r) {  // eliminate column i everywhere (Gauss-Jordan)
            const int e = mat[r * n + i];
            if (r == i || e == 0) continue;
            for (int c = 0; c < n; ++c) {
                mat[r * n + c] ^= gf_mul(e, mat[i * n + c]);
                inv[r * n + c] ^= gf_mul(e, inv[i * n + c]);
            }
        }
    }
    return 0;
}

}  // namespace cec
