// ambrycrc_chain_messages_host (the sequential header hop of BlobStoreRecovery.recover) under
// AddressSanitizer + UBSan: it parses untrusted log bytes, so it is run from every start offset
// of a region and on every truncation of its tail, each time on an exactly-sized copy, so a
// read past the region is caught. Host code only (no HIP call is made). Reads the region file
// written by tests/test_abi.py; prints the number of runs.
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "../../include/ambrycrc.h"

int main(int argc, char** argv) {
  if (argc < 2) return 2;
  FILE* f = fopen(argv[1], "rb");
  if (!f) return 2;
  std::vector<unsigned char> all;
  unsigned char buf[65536];
  size_t got;
  while ((got = fread(buf, 1, sizeof buf, f)) > 0) all.insert(all.end(), buf, buf + got);
  fclose(f);
  std::vector<uint64_t> offs(1 << 16);
  long runs = 0;
  // every start offset of the first 6000 bytes, full region
  for (size_t start = 0; start < 6000 && start < all.size(); ++start) {
    unsigned char* r = (unsigned char*)malloc(all.size());
    memcpy(r, all.data(), all.size());
    (void)ambrycrc_chain_messages_host(r, all.size(), start, offs.data(), offs.size());
    free(r);
    ++runs;
  }
  // every truncation of the last 6000 bytes
  for (size_t cut = all.size() > 6000 ? all.size() - 6000 : 0; cut <= all.size(); ++cut) {
    unsigned char* r = (unsigned char*)malloc(cut ? cut : 1);
    memcpy(r, all.data(), cut);
    (void)ambrycrc_chain_messages_host(r, cut, 0, offs.data(), offs.size());
    free(r);
    ++runs;
  }
  printf("runs=%ld\n", runs);
  return 0;
}
