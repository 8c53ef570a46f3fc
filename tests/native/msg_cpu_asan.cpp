// ambrycrc_verify_message_cpu / ambrycrc_transform_message_cpu under AddressSanitizer + UBSan:
// they parse untrusted log bytes, so each message of the region (written by tests/test_abi.py)
// is run on an exactly-sized copy, on every truncation of it, and with random bytes of its
// header and record heads (versions, size fields, offsets) flipped; the transform's output
// buffer is sized exactly to what the call may write. Host code only (no HIP call is made).
// Prints the number of runs.
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "../../include/ambrycrc.h"

static void run(const std::vector<unsigned char>& msg, long* runs) {
  unsigned char* r = (unsigned char*)malloc(msg.size() ? msg.size() : 1);
  if (!msg.empty()) memcpy(r, msg.data(), msg.size());
  uint32_t st = 0;
  uint64_t end = 0, n = 0;
  (void)ambrycrc_verify_message_cpu(r, msg.size(), 0, &st, &end);
  const uint64_t cap = msg.size() + 16;
  unsigned char* out = (unsigned char*)malloc(cap);
  for (int v = 1; v <= 3; ++v) (void)ambrycrc_transform_message_cpu(r, msg.size(), 0, -1, v, out, cap, &n, &st);
  free(out);
  free(r);
  ++*runs;
}

int main(int argc, char** argv) {
  if (argc < 2) return 2;
  FILE* f = fopen(argv[1], "rb");
  if (!f) return 2;
  std::vector<unsigned char> all;
  unsigned char buf[65536];
  size_t got;
  while ((got = fread(buf, 1, sizeof buf, f)) > 0) all.insert(all.end(), buf, buf + got);
  fclose(f);
  std::vector<uint64_t> offs(4096);
  const size_t m = ambrycrc_chain_messages_host(all.data(), all.size(), 0, offs.data(), offs.size());
  long runs = 0;
  uint64_t rng = 0x9E3779B97F4A7C15ull;
  for (size_t i = 0; i < m; ++i) {
    const size_t lo = offs[i], hi = i + 1 < m ? offs[i + 1] : all.size();
    std::vector<unsigned char> msg(all.begin() + lo, all.begin() + hi);
    run(msg, &runs);
    for (size_t cut = 0; cut < msg.size(); cut += 1 + cut / 8) run(std::vector<unsigned char>(msg.begin(), msg.begin() + cut), &runs);
    for (int t = 0; t < 300; ++t) {  // flips in the header and record heads: the first 64 bytes, then the first 320
      std::vector<unsigned char> bad(msg);
      const size_t span = t < 200 ? 64 : 320;  // (the properties record's int-length strings sit past byte 64)
      for (int k = 0; k < 3; ++k) {
        rng = rng * 6364136223846793005ull + 1442695040888963407ull;
        const size_t at = (size_t)(rng >> 33) % (bad.size() < span ? bad.size() : span);
        bad[at] ^= (unsigned char)(1u << ((rng >> 20) & 7));
      }
      run(bad, &runs);
    }
  }
  printf("runs=%ld messages=%zu\n", runs, m);
  return m ? 0 : 1;
}
