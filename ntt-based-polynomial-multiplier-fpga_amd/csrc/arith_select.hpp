// arith_select.hpp — which 32-bit arithmetic class handles a modulus q < 2^32.  Shared by the
// planner (the twiddle-pair format it emits) and the kernel dispatch (the class that consumes it),
// so the two cannot disagree.
#pragma once
#include <stdint.h>

// Arith32H (Harvey bounds, Montgomery-form twiddles) for q < 2^30
#ifndef NTTMUL_A32H
#define NTTMUL_A32H 1
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

namespace nttmul {

enum class A32Kind { Harvey, Plantard, Mont, Wide };

// q < 2^32 only (64-bit words take Arith64)
constexpr A32Kind a32_kind(uint64_t q) {
  return NTTMUL_A32H && q < (1ull << 30)      ? A32Kind::Harvey
         : q >= (1ull << 31)                  ? A32Kind::Wide
         : NTTMUL_A32_PLANTARD                ? A32Kind::Plantard
                                              : A32Kind::Mont;
}

}  // namespace nttmul
