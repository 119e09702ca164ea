// Standalone self-test of the native runtime, built with AddressSanitizer + UBSan by
// tools/sanitize_rt.sh (race/memory checking of host code; GPU sanitizers are not
// available on this pool).  Exercises every parser on valid AND corrupted / truncated inputs, so
// out-of-bounds reads in the SSTable / proto / TFRecord / CIFAR code paths are caught.
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <random>
#include <string>
#include <vector>

#include "../rt.h"

using namespace dmlc_rt;

static int failures = 0;
#define EXPECT(c)                                                      \
  do {                                                                 \
    if (!(c)) {                                                        \
      std::fprintf(stderr, "FAILED %s:%d: %s\n", __FILE__, __LINE__, #c); \
      ++failures;                                                      \
    }                                                                  \
  } while (0)

int main(int argc, char** argv) {
  const std::string dir = argc > 1 ? argv[1] : "/tmp";
  std::mt19937 rng(1234);

  // crc32c check value
  const char* check = "123456789";
  EXPECT(crc32c((const uint8_t*)check, 9) == 0xE3069283u);
  EXPECT(crc_unmask(crc_mask(0xdeadbeefu)) == 0xdeadbeefu);

  // tables: many sizes / block sizes; then every truncation and random bit flips must fail cleanly
  for (int n : {0, 1, 5, 40, 300}) {
    for (size_t bs : {64, 4096, 262144}) {
      TableBuilder tb(bs, 16);
      std::vector<std::pair<std::string, std::string>> want;
      for (int i = 0; i < n; ++i) {
        char k[32];
        std::snprintf(k, sizeof(k), "key/%06d", i);
        std::string v(rng() % 100, (char)(rng() & 0xff));
        tb.add(k, v);
        want.emplace_back(k, v);
      }
      const std::string img = tb.finish();
      std::vector<std::pair<std::string, std::string>> got;
      std::string err;
      EXPECT(read_table(img, &got, &err));
      EXPECT(got == want);
      for (size_t cut = 0; cut < img.size(); cut += 1 + img.size() / 50) {
        std::vector<std::pair<std::string, std::string>> kv;
        (void)read_table(img.substr(0, cut), &kv, &err);     // must not crash / over-read
      }
      for (int f = 0; f < 50 && !img.empty(); ++f) {
        std::string bad = img;
        bad[rng() % bad.size()] ^= (char)(1 << (rng() % 8));
        std::vector<std::pair<std::string, std::string>> kv;
        (void)read_table(bad, &kv, &err);
      }
    }
  }

  // bundle round trip + corrupted entry protos
  {
    const std::string prefix = dir + "/rt_selftest.ckpt";
    std::vector<std::string> names = {"b", "a/w", "global_step"};
    std::vector<int> dt = {DT_FLOAT, DT_FLOAT, DT_INT64};
    std::vector<std::vector<int64_t>> shapes = {{3}, {2, 2}, {}};
    std::vector<std::string> data = {std::string(12, 'x'), std::string(16, 'y'), std::string(8, 'z')};
    EXPECT(write_bundle(prefix, names, dt, shapes, data).empty());
    std::vector<BundleEntry> ents;
    std::vector<std::string> blobs;
    EXPECT(read_bundle(prefix, &ents, &blobs).empty());
    EXPECT(ents.size() == 3 && ents[0].name == "a/w" && blobs[0] == data[1]);
    EXPECT(!write_bundle(prefix, {"x"}, {DT_FLOAT}, {{2}}, {std::string(7, 'q')}).empty());   // size mismatch
    for (int f = 0; f < 200; ++f) {
      BundleEntry e;
      e.dtype = DT_FLOAT; e.shape = {(int64_t)(rng() % 9), 3}; e.size = 36; e.offset = rng() % 1000;
      std::string enc = encode_entry(e);
      enc.resize(rng() % (enc.size() + 1));
      if (!enc.empty() && (rng() & 1)) enc[rng() % enc.size()] ^= 0x80;
      BundleEntry d;
      std::string err;
      (void)decode_entry(enc, &d, &err);
    }
  }

  // TFRecord framing
  {
    const std::string ev = encode_event_scalars(1.5, 42, {"loss", "acc"}, {0.5f, 0.25f});
    const std::string rec = tfrecord_frame(ev);
    EXPECT(rec.size() == ev.size() + 16);
    EXPECT(get_fixed64((const uint8_t*)rec.data()) == ev.size());
  }

  // CIFAR reader: valid file, truncated file, empty list
  {
    const std::string f = dir + "/rt_selftest_batch.bin";
    std::string buf(3073 * 3, '\0');
    for (int r = 0; r < 3; ++r) {
      buf[r * 3073] = (char)(r + 1);
      for (int i = 0; i < 3072; ++i) buf[r * 3073 + 1 + i] = (char)((i + r) & 0xff);
    }
    std::ofstream(f, std::ios::binary).write(buf.data(), (std::streamsize)buf.size());
    std::vector<uint8_t> img;
    std::vector<int32_t> lab;
    EXPECT(read_cifar_files({f, f}, &img, &lab, 4).empty());
    EXPECT(lab.size() == 6 && lab[4] == 2 && img.size() == 6 * 3072u);
    EXPECT(img[3072 + 1] == (uint8_t)((1024 + 1) & 0xff));      // pixel 0, channel 1 of record 1
    std::ofstream(f, std::ios::binary).write(buf.data(), 3000);
    EXPECT(!read_cifar_files({f}, &img, &lab, 2).empty());
    EXPECT(read_cifar_files({}, &img, &lab, 2).empty() && lab.empty());
  }

  std::printf("rt_selftest: %s (%d failure(s))\n", failures ? "FAILED" : "ok", failures);
  return failures ? 1 : 0;
}
