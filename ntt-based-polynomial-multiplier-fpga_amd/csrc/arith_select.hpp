// arith_select.hpp — which 32-bit arithmetic class handles a modulus q < 2^32.  Shared by the
// planner (the twiddle-pair format it emits) and the kernel dispatch (the class that consumes it),
// so the two cannot disagree.
#pragma once
#include <stdint.h>

// Arith32H (Harvey bounds, Montgomery-form twiddles) for q < 2^30 (1); 0 = those q take Arith32P
// as well (round 2: the Plantard kernels' bounds hold for every q < 2^31, and at q = 1073479681
// they run n = 4096 products 9 % and n = 1024 products 7 % faster than Arith32H, kbench A/B
// in profiles/r2/a32h_ab.txt)
#ifndef NTTMUL_A32H
#define NTTMUL_A32H 0
#endif
// Arith32P (Plantard twiddle products, canonical output for any 32-bit input) for the q < 2^31
// not taken by Arith32H; 0 = the Montgomery Arith32 with typed butterflies (round-1 kernel)
#ifndef NTTMUL_A32_PLANTARD
#define NTTMUL_A32_PLANTARD 1
#endif

// Arith32P inverse twiddles in the signed-input Plantard form (the GS difference x - y in (-q, q)
// is multiplied without "+ q"); planner and kernels must agree
#ifndef NTTMUL_P_SIGNED_INV
#define NTTMUL_P_SIGNED_INV 1
#endif

// column stages of the n = 65536 multi-pass product (4: 16 x 4096 rows, 5: 32 x 2048)
#ifndef NTTMUL_SPLIT16
#define NTTMUL_SPLIT16 4
#endif
// 64-bit words at n = 65536 (C5): the square split 256 x 256 (kernels_dev.hpp k_cols8; 8 column
// stages in the HBM-bound column passes, 8 in the row pass) instead of NTTMUL_SPLIT16's.  The
// 32-bit classes keep NTTMUL_SPLIT16 (their twiddle typing, p_signed_fw_entry, follows it)
#ifndef NTTMUL_C5_SQ
#define NTTMUL_C5_SQ 1
#endif
// Arith32P forward CT typing: 0 = off; 1 = a difference x - t stays signed when its next use in
// the register group is as an X; 2 = every in-group difference stays signed and is multiplied by
// the signed-input Plantard product, so the planner stores those forward twiddles in signed form
// (p_signed_fw_entry); planner and kernels must agree
#ifndef NTTMUL_P_TYPED
#define NTTMUL_P_TYPED 2
#endif

namespace nttmul {

// log2 of the rows a product / transform runs in registers + LDS (kernels.hip k_rows, k_xform):
// the whole polynomial up to n = 4096, else 4096-coefficient rows after L1 = logn - LOGS column
// stages
constexpr int row_logs(int logn) {
  return logn <= 12 ? logn : (logn == 16 && NTTMUL_SPLIT16 == 5 ? 11 : 12);
}
// register groups of a row of 2^LOGS coefficients (kernels.hip Groups<LOGS>::G / S / ST0)
constexpr int groups_g(int logs) { return (logs + 3) / 4; }
constexpr int groups_s(int logs, int g) {
  return logs / groups_g(logs) + (g < logs % groups_g(logs) ? 1 : 0);
}
// Wave-typed register-group layouts of the Plantard kernels' 4096-coefficient rows (kernels.hip
// Groups WT); planner and kernels must agree.  Off: C3 +2.0 % time (1.034 vs 1.013 ms, kbench
// A/B, identical checksums, profiles/r3/c3/wave_typed_ab.txt) -- the permuted layouts' address
// math and the branch's join copies cost more than the 32 boundary instructions they remove
#ifndef NTTMUL_WAVE_TYPED
#define NTTMUL_WAVE_TYPED 0
#endif
constexpr bool wave_typed_rows(int logs) { return NTTMUL_WAVE_TYPED && logs == 12; }
// Arith32P, NTTMUL_P_TYPED == 2: forward twiddle entry idx = 2^st + j serves stage st; at a
// stage that is not the first of its register group, the multiplicand of the butterflies using
// an odd entry is the previous stage's difference (bit 2d of the element = the entry's low bit),
// kept signed: that entry is stored in the signed-input form
constexpr bool p_signed_fw_entry(int logn, uint32_t idx) {
  if (idx < 2) return false;
  int st = 0;
  while ((2u << st) <= idx) st++;
  const int logs = row_logs(logn), local = st - (logn - logs);
  if (local < 0) return false;  // column pass: unsigned operands
  int g = 0, st0 = 0;
  while (st0 + groups_s(logs, g) <= local) st0 += groups_s(logs, g++);
  // wave-typed layouts (kernels.hip Groups WT, 4096-coefficient rows): the first stage of groups
  // 1 and 2 multiplies the previous group's differences, left signed across the exchange, by the
  // odd entries as well
  return (local - st0 >= 1 || (wave_typed_rows(logs) && g >= 1)) && (idx & 1);
}

// Arith32P3 (base blocks of 8 coefficients, n = 4096 products only): each output sums eight
// products of canonical values; the first four are folded by 2^32 mod q before the other four
// are added.  With q = x 2^31 the sum is below x^2 (2 - x) 2^64 when 2^32 mod q = 2^32 - 2q
// (x > 2/3) and below x^2 (2 - 1.5 x) 2^64 when it is 2^32 - 3q, so every 2^30 < q < 2^31
// qualifies; below 2^30 the first four products stay under 2^62 and the fold under 2^62 + 2^32.
// The check is kept so a change of range cannot silently overflow
#ifndef NTTMUL_P3
#define NTTMUL_P3 1
#endif
constexpr bool p3_fold_ok(uint64_t q) {
  if (!NTTMUL_P3 || q >= (1ull << 31) || q < 3) return false;
  const unsigned __int128 s1 = (unsigned __int128)4 * (q - 1) * (q - 1);  // < 2^64
  const unsigned __int128 c32 = ((unsigned __int128)1 << 32) % q;
  const unsigned __int128 fold = (s1 >> 32) * c32 + 0xFFFFFFFFu;
  return fold + s1 < ((unsigned __int128)1 << 64);
}

enum class A32Kind { Harvey, Plantard, Mont, Wide };

// q < 2^32 only (64-bit words take Arith64)
constexpr A32Kind a32_kind(uint64_t q) {
  return NTTMUL_A32H && q < (1ull << 30)      ? A32Kind::Harvey
         : q >= (1ull << 31)                  ? A32Kind::Wide
         : NTTMUL_A32_PLANTARD                ? A32Kind::Plantard
                                              : A32Kind::Mont;
}

}  // namespace nttmul
