// CRC32C (Castagnoli) for the LevelDB codec (sparknet_amd/data/leveldb.py): block
// trailers and log records of every table / log file carry a masked CRC32C.  Uses the
// SSE4.2 crc32 instruction (8 bytes per step) when the CPU has it, a table otherwise.
#include <cstddef>
#include <cstdint>
#include <cstring>

namespace {

uint32_t g_table[256];
bool g_init = false;

void init_table() {
  for (uint32_t i = 0; i < 256; ++i) {
    uint32_t c = i;
    for (int k = 0; k < 8; ++k) c = (c & 1) ? (c >> 1) ^ 0x82F63B78u : c >> 1;
    g_table[i] = c;
  }
  g_init = true;
}

uint32_t crc_table(const uint8_t* p, size_t n, uint32_t crc) {
  if (!g_init) init_table();
  for (size_t i = 0; i < n; ++i) crc = g_table[(crc ^ p[i]) & 0xFF] ^ (crc >> 8);
  return crc;
}

__attribute__((target("sse4.2"))) uint32_t crc_hw(const uint8_t* p, size_t n, uint32_t crc) {
  uint64_t c = crc;
  while (n >= 8) {
    uint64_t v;
    std::memcpy(&v, p, 8);
    c = __builtin_ia32_crc32di(c, v);
    p += 8;
    n -= 8;
  }
  uint32_t c32 = static_cast<uint32_t>(c);
  while (n--) c32 = __builtin_ia32_crc32qi(c32, *p++);
  return c32;
}

}  // namespace

extern "C" uint32_t sn_crc32c(const void* data, size_t n, uint32_t init) {
  const uint8_t* p = static_cast<const uint8_t*>(data);
  uint32_t crc = ~init;
  crc = __builtin_cpu_supports("sse4.2") ? crc_hw(p, n, crc) : crc_table(p, n, crc);
  return ~crc;
}
