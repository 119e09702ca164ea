// crc32c (Castagnoli, reflected 0x82F63B78) + little-endian / varint coding.
// Slicing-by-8 table implementation; the SSE4.2 crc32 instruction is used when the host has it.
#include "rt.h"

#include <cstring>
#if defined(__x86_64__)
#include <cpuid.h>
#include <nmmintrin.h>
#endif

namespace dmlc_rt {

namespace {

struct Tables {
  uint32_t t[8][256];
  Tables() {
    for (uint32_t i = 0; i < 256; ++i) {
      uint32_t c = i;
      for (int k = 0; k < 8; ++k) c = (c >> 1) ^ (0x82F63B78u & (0u - (c & 1u)));
      t[0][i] = c;
    }
    for (uint32_t i = 0; i < 256; ++i)
      for (int s = 1; s < 8; ++s) t[s][i] = (t[s - 1][i] >> 8) ^ t[0][t[s - 1][i] & 0xff];
  }
};
const Tables& tables() {
  static const Tables tb;
  return tb;
}

uint32_t crc_sw(uint32_t c, const uint8_t* p, size_t n) {
  const Tables& T = tables();
  while (n >= 8) {
    uint64_t w;
    std::memcpy(&w, p, 8);
    w ^= c;
    c = T.t[7][w & 0xff] ^ T.t[6][(w >> 8) & 0xff] ^ T.t[5][(w >> 16) & 0xff] ^ T.t[4][(w >> 24) & 0xff] ^
        T.t[3][(w >> 32) & 0xff] ^ T.t[2][(w >> 40) & 0xff] ^ T.t[1][(w >> 48) & 0xff] ^ T.t[0][w >> 56];
    p += 8;
    n -= 8;
  }
  while (n--) c = (c >> 8) ^ T.t[0][(c ^ *p++) & 0xff];
  return c;
}

#if defined(__x86_64__)
__attribute__((target("sse4.2"))) uint32_t crc_hw(uint32_t c, const uint8_t* p, size_t n) {
  uint64_t c64 = c;
  while (n >= 8) {
    uint64_t w;
    std::memcpy(&w, p, 8);
    c64 = _mm_crc32_u64(c64, w);
    p += 8;
    n -= 8;
  }
  uint32_t c32 = (uint32_t)c64;
  while (n--) c32 = _mm_crc32_u8(c32, *p++);
  return c32;
}
bool have_sse42() {
  unsigned a, b, cc, d;
  if (!__get_cpuid(1, &a, &b, &cc, &d)) return false;
  return (cc & bit_SSE4_2) != 0;
}
#endif

}  // namespace

uint32_t crc32c_extend(uint32_t crc, const uint8_t* data, size_t n) {
  uint32_t c = ~crc;
#if defined(__x86_64__)
  static const bool hw = have_sse42();
  c = hw ? crc_hw(c, data, n) : crc_sw(c, data, n);
#else
  c = crc_sw(c, data, n);
#endif
  return ~c;
}

void put_fixed32(std::string* dst, uint32_t v) {
  char b[4];
  for (int i = 0; i < 4; ++i) b[i] = (char)((v >> (8 * i)) & 0xff);
  dst->append(b, 4);
}

void put_fixed64(std::string* dst, uint64_t v) {
  char b[8];
  for (int i = 0; i < 8; ++i) b[i] = (char)((v >> (8 * i)) & 0xff);
  dst->append(b, 8);
}

void put_varint(std::string* dst, uint64_t v) {
  while (v >= 0x80) {
    dst->push_back((char)((v & 0x7f) | 0x80));
    v >>= 7;
  }
  dst->push_back((char)v);
}

uint32_t get_fixed32(const uint8_t* p) {
  return (uint32_t)p[0] | ((uint32_t)p[1] << 8) | ((uint32_t)p[2] << 16) | ((uint32_t)p[3] << 24);
}

uint64_t get_fixed64(const uint8_t* p) { return (uint64_t)get_fixed32(p) | ((uint64_t)get_fixed32(p + 4) << 32); }

const uint8_t* get_varint(const uint8_t* p, const uint8_t* end, uint64_t* v) {
  uint64_t r = 0;
  for (int shift = 0; shift <= 63 && p < end; shift += 7) {
    const uint8_t b = *p++;
    r |= (uint64_t)(b & 0x7f) << shift;
    if (!(b & 0x80)) {
      *v = r;
      return p;
    }
  }
  return nullptr;
}

}  // namespace dmlc_rt
