// pcie_shim.cpp — lib/terasic_pcie_qsys.so: the Terasic PCIe driver ABI that the reference's
// FPGA communicator loads (Software_Hardware_Comunnicator/linux_app/PCIE.c:59-103 dlopens
// "./terasic_pcie_qsys.so" and resolves 12 symbols), implemented on top of libnttmul so that
// NTT_PCIECommunicationv2.c runs UNCHANGED with the MI355X in place of the DE2i-150 board.
// SURVEY §8f row 3 (FPGA-compat).
//
// Emulated device (the PolyMult FSM as the communicator drives it, NTT_PCIECommunicationv2.c):
//   BAR0 + 0x00 (ADDR_CONTROL) write: bit 0 = start, bits [3:1] = mode            (:43-51)
//   BAR0 + 0x20 (ADDR_STATUS)  read : bit 0 = busy, bit 1 = done_all                (:24-25)
//   FIFO 0x40 (FIFO_IN)  DMA write: mode 0 -> W[W_COUNT], W_INV[W_COUNT], q, n_inv  (:140-148)
//                                   mode 1 -> A[256], mode 2 -> B[256]              (:183-202)
//   mode 3 start (GO): c = a * b mod (x^256 - 1, q) on the GPU, then done_all = 1   (:211-215)
//   FIFO 0x80 (FIFO_OUT) DMA read : C[256]                                          (:220-224)
// The product is the RTL's cyclic convolution (Hardware_Multiplier/PolyMult.v, verified against
// the reference's ModelSim vectors in tests/).  q and omega come from the mode-0 stream itself:
// W[0] = w^0 R = R mod q and W[1] = w R mod q (generate_params.C:54-73), so omega = W[1] / W[0].
// (The committed RTL hard-wires q = 7681 in its pointwise unit, PolyMult.v:282, while the v2
// communicator streams q = 12289; the emulation follows the stream.)
// Plain Read/Write 8/16/32 to other addresses and DmaRead/DmaWrite hit a 64 KiB scratch RAM.
#include <stdint.h>
#include <stdio.h>
#include <string.h>

#include <map>
#include <mutex>
#include <vector>

#include "nttmul.h"
#include "planner.hpp"

namespace {

constexpr uint32_t kN = 256;               // RING_SIZE (Hardware_Multiplier/defines.v:26)
constexpr uint32_t kPE = 8;                // PE_NUMBER (defines.v:27)
constexpr uint32_t kAddrControl = 0x00, kAddrStatus = 0x20;
constexpr uint32_t kFifoIn = 0x40, kFifoOut = 0x80;

struct Board {
  uint32_t mode = 0, busy = 0, done = 0;
  std::vector<uint32_t> params, a, b, c;
  size_t expect = 0;                       // words the current mode still waits for
  std::vector<uint8_t> ram = std::vector<uint8_t>(65536, 0);
  std::map<std::pair<uint64_t, uint64_t>, nttmul_ctx *> ctx;  // (q, omega) -> cyclic context
  char err[256] = {0};
};

std::mutex g_mu;
std::map<int, Board *> g_boards;
int g_next = 1;

size_t w_count() {  // generate_twiddles stream length for N = 256, PE = 8 (272)
  return nttmul_fpga_twiddles(kN, 3, 1, 1, kPE, nullptr, 0);
}

Board *board(int h) {
  auto it = g_boards.find(h);
  return it == g_boards.end() ? nullptr : it->second;
}

bool go(Board *B) {
  const size_t wc = w_count();
  if (B->params.size() < 2 * wc + 2 || B->a.size() < kN || B->b.size() < kN) {
    snprintf(B->err, sizeof(B->err), "GO before modes 0/1/2 completed");
    return false;
  }
  const uint64_t q = B->params[2 * wc];
  if (q < 3 || !nttmul_is_prime(q)) {  // before any "% q": q = 0 from the stream must not trap
    snprintf(B->err, sizeof(B->err), "mode-0 stream: q = %llu is not an odd prime",
             (unsigned long long)q);
    return false;
  }
  const uint64_t r = B->params[0] % q, wr = B->params[1] % q;
  if (!r) return false;
  // the board multiplies whatever the FIFOs delivered: reduce A and B into [0, q) as its
  // modular datapath does, so the validated-input contract of nttmul_multiply holds
  for (uint32_t i = 0; i < kN; i++) {
    B->a[i] = (uint32_t)(B->a[i] % q);
    B->b[i] = (uint32_t)(B->b[i] % q);
  }
  const uint64_t omega = nttmul::mulmod(wr, nttmul::powmod(r, q - 2, q), q);
  nttmul_ctx *&ctx = B->ctx[{q, omega}];
  if (!ctx) {
    nttmul_params p = {kN, q, omega, 1, 0, NTTMUL_FLAG_CYCLIC};
    int st = nttmul_create_ex(&ctx, &p);
    if (st) {
      snprintf(B->err, sizeof(B->err), "nttmul_create_ex: %s", nttmul_strerror(st));
      ctx = nullptr;
      return false;
    }
  }
  B->c.assign(kN, 0);
  int st = nttmul_multiply_u32(ctx, B->c.data(), B->a.data(), B->b.data());
  if (st) snprintf(B->err, sizeof(B->err), "nttmul_multiply_u32: %s", nttmul_strerror(st));
  return st == 0;
}

}  // namespace

extern "C" {

int PCIE_Open(unsigned short, unsigned short, unsigned short) {
  nttmul_ctx *probe = nullptr;
  if (nttmul_create(&probe, kN, 12289, 1) != NTTMUL_OK) return 0;  // no usable GPU
  nttmul_destroy(probe);
  std::lock_guard<std::mutex> l(g_mu);
  g_boards[g_next] = new Board();
  return g_next++;
}

void PCIE_Close(int h) {
  std::lock_guard<std::mutex> l(g_mu);
  Board *B = board(h);
  if (!B) return;
  for (auto &kv : B->ctx) nttmul_destroy(kv.second);
  delete B;
  g_boards.erase(h);
}

int PCIE_Write32(int h, int bar, unsigned int addr, unsigned int data) {
  std::lock_guard<std::mutex> l(g_mu);
  Board *B = board(h);
  if (!B) return 0;
  if (bar == 0 && addr == kAddrControl) {
    if (data & 1) {  // start pulse
      B->mode = (data >> 1) & 7;
      B->done = 0;
      switch (B->mode) {
        case 0: B->params.clear(); B->expect = 2 * w_count() + 2; B->busy = 1; break;
        case 1: B->a.clear(); B->expect = kN; B->busy = 1; break;
        case 2: B->b.clear(); B->expect = kN; B->busy = 1; break;
        case 3: B->busy = 1; B->done = go(B) ? 1 : 0; B->busy = 0; break;
        default: break;
      }
    }
    return 1;
  }
  if ((size_t)addr + 4 > B->ram.size()) return 0;
  memcpy(&B->ram[addr], &data, 4);
  return 1;
}

int PCIE_Read32(int h, int bar, unsigned int addr, unsigned int *data) {
  std::lock_guard<std::mutex> l(g_mu);
  Board *B = board(h);
  if (!B || !data) return 0;
  if (bar == 0 && addr == kAddrStatus) {
    *data = (B->busy & 1) | ((B->done & 1) << 1);
    return 1;
  }
  if ((size_t)addr + 4 > B->ram.size()) return 0;
  memcpy(data, &B->ram[addr], 4);
  return 1;
}

int PCIE_Write16(int h, int, unsigned int addr, unsigned short v) {
  std::lock_guard<std::mutex> l(g_mu);
  Board *B = board(h);
  if (!B || (size_t)addr + 2 > B->ram.size()) return 0;
  memcpy(&B->ram[addr], &v, 2);
  return 1;
}
int PCIE_Read16(int h, int, unsigned int addr, unsigned short *v) {
  std::lock_guard<std::mutex> l(g_mu);
  Board *B = board(h);
  if (!B || !v || (size_t)addr + 2 > B->ram.size()) return 0;
  memcpy(v, &B->ram[addr], 2);
  return 1;
}
int PCIE_Write8(int h, int, unsigned int addr, unsigned char v) {
  std::lock_guard<std::mutex> l(g_mu);
  Board *B = board(h);
  if (!B || addr >= B->ram.size()) return 0;
  B->ram[addr] = v;
  return 1;
}
int PCIE_Read8(int h, int, unsigned int addr, unsigned char *v) {
  std::lock_guard<std::mutex> l(g_mu);
  Board *B = board(h);
  if (!B || !v || addr >= B->ram.size()) return 0;
  *v = B->ram[addr];
  return 1;
}
int PCIE_DmaWrite(int h, unsigned int addr, void *p, unsigned int n) {
  std::lock_guard<std::mutex> l(g_mu);
  Board *B = board(h);
  if (!B || !p || (size_t)addr + n > B->ram.size()) return 0;
  memcpy(&B->ram[addr], p, n);
  return 1;
}
int PCIE_DmaRead(int h, unsigned int addr, void *p, unsigned int n) {
  std::lock_guard<std::mutex> l(g_mu);
  Board *B = board(h);
  if (!B || !p || (size_t)addr + n > B->ram.size()) return 0;
  memcpy(p, &B->ram[addr], n);
  return 1;
}

int PCIE_DmaFifoWrite(int h, unsigned int fifo, void *p, unsigned int n) {
  std::lock_guard<std::mutex> l(g_mu);
  Board *B = board(h);
  if (!B || !p || fifo != kFifoIn || n % 4) return 0;
  const uint32_t *w = (const uint32_t *)p;
  std::vector<uint32_t> *dst = B->mode == 0 ? &B->params : B->mode == 1 ? &B->a
                             : B->mode == 2 ? &B->b : nullptr;
  if (!dst) return 0;
  dst->insert(dst->end(), w, w + n / 4);
  B->expect = B->expect > n / 4 ? B->expect - n / 4 : 0;
  if (!B->expect) B->busy = 0;
  return 1;
}

int PCIE_DmaFifoRead(int h, unsigned int fifo, void *p, unsigned int n) {
  std::lock_guard<std::mutex> l(g_mu);
  Board *B = board(h);
  if (!B || !p || fifo != kFifoOut || !B->done || n > B->c.size() * 4) return 0;
  memcpy(p, B->c.data(), n);
  return 1;
}

}  // extern "C"
