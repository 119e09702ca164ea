// TFRecord framing + tf.Event encoding (the chief's events.out.tfevents.* file of TF1's
// MonitoredTrainingSession summaries, /root/reference/cifar10cnn.py:222) and the
// CIFAR-10 binary reader (FixedLengthRecordReader(3073) + decode_raw + CHW->HWC,
// cifar10cnn.py:54-66).
#include "rt.h"

#include <fcntl.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>

#include <cstring>
#include <thread>
#include <algorithm>

namespace dmlc_rt {

std::string tfrecord_frame(const std::string& payload) {
  std::string out, len;
  put_fixed64(&len, payload.size());
  out.append(len);
  put_fixed32(&out, crc_mask(crc32c((const uint8_t*)len.data(), len.size())));
  out.append(payload);
  put_fixed32(&out, crc_mask(crc32c((const uint8_t*)payload.data(), payload.size())));
  return out;
}

namespace {
void put_double_field(std::string* s, int field, double v) {
  put_varint(s, (uint64_t)((field << 3) | 1));
  uint64_t bits;
  std::memcpy(&bits, &v, 8);
  put_fixed64(s, bits);
}
void put_string_field(std::string* s, int field, const std::string& v) {
  put_varint(s, (uint64_t)((field << 3) | 2));
  put_varint(s, v.size());
  s->append(v);
}
}  // namespace

// Event { double wall_time = 1; int64 step = 2; oneof what { string file_version = 3; Summary summary = 5; } }
std::string encode_event_file_version(double wall_time) {
  std::string s;
  put_double_field(&s, 1, wall_time);
  put_string_field(&s, 3, "brain.Event:2");
  return s;
}

// Summary { repeated Value value = 1; }  Value { string tag = 1; float simple_value = 2; }
std::string encode_event_scalars(double wall_time, int64_t step, const std::vector<std::string>& tags,
                                 const std::vector<float>& values) {
  std::string summary;
  for (size_t i = 0; i < tags.size() && i < values.size(); ++i) {
    std::string v;
    put_string_field(&v, 1, tags[i]);
    put_varint(&v, (2 << 3) | 5);
    uint32_t bits;
    std::memcpy(&bits, &values[i], 4);
    put_fixed32(&v, bits);
    put_string_field(&summary, 1, v);
  }
  std::string s;
  put_double_field(&s, 1, wall_time);
  if (step) {
    put_varint(&s, (2 << 3) | 0);
    put_varint(&s, (uint64_t)step);
  }
  put_string_field(&s, 5, summary);
  return s;
}

std::string read_cifar_files(const std::vector<std::string>& files, std::vector<uint8_t>* images,
                             std::vector<int32_t>* labels, int threads) {
  constexpr size_t kRec = 3073, kImg = 3072;
  struct Map {
    const uint8_t* p = nullptr;
    size_t n = 0;
    int fd = -1;
  };
  std::vector<Map> maps;
  size_t total = 0;
  auto unmap_all = [&]() {
    for (auto& m : maps) {
      if (m.p) munmap((void*)m.p, m.n);
      if (m.fd >= 0) close(m.fd);
    }
  };
  for (const auto& f : files) {
    Map m;
    m.fd = open(f.c_str(), O_RDONLY);
    if (m.fd < 0) { unmap_all(); return "cannot open " + f; }
    struct stat st;
    if (fstat(m.fd, &st) != 0) { close(m.fd); unmap_all(); return "cannot stat " + f; }
    m.n = (size_t)st.st_size;
    if (m.n % kRec != 0) { close(m.fd); unmap_all(); return f + ": size is not a multiple of 3073-byte records"; }
    if (m.n) {
      void* p = mmap(nullptr, m.n, PROT_READ, MAP_PRIVATE, m.fd, 0);
      if (p == MAP_FAILED) { close(m.fd); unmap_all(); return "cannot mmap " + f; }
      madvise(p, m.n, MADV_SEQUENTIAL);
      m.p = (const uint8_t*)p;
    }
    maps.push_back(m);
    total += m.n / kRec;
  }
  images->resize(total * kImg);
  labels->resize(total);
  std::vector<std::pair<const uint8_t*, size_t>> recs;  // (file base, first global record)
  size_t g = 0;
  for (auto& m : maps) {
    recs.emplace_back(m.p, g);
    g += m.n / kRec;
  }
  threads = std::max(1, std::min(threads, 64));
  auto work = [&](size_t r0, size_t r1) {
    size_t fi = 0;
    for (size_t r = r0; r < r1; ++r) {
      while (fi + 1 < recs.size() && r >= recs[fi + 1].second) ++fi;
      const uint8_t* src = recs[fi].first + (r - recs[fi].second) * kRec;
      (*labels)[r] = (int32_t)src[0];
      const uint8_t* chw = src + 1;
      uint8_t* dst = images->data() + r * kImg;
      for (int p = 0; p < 1024; ++p) {   // CHW [3][32][32] -> HWC [32][32][3]
        dst[3 * p + 0] = chw[p];
        dst[3 * p + 1] = chw[1024 + p];
        dst[3 * p + 2] = chw[2048 + p];
      }
    }
  };
  std::vector<std::thread> pool;
  const size_t per = (total + threads - 1) / threads;
  for (int t = 0; t < threads; ++t) {
    const size_t r0 = t * per, r1 = std::min(total, r0 + per);
    if (r0 >= r1) break;
    pool.emplace_back(work, r0, r1);
  }
  for (auto& th : pool) th.join();
  unmap_all();
  return "";
}

}  // namespace dmlc_rt
