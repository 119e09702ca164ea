// Native CPU runtime of the framework (no torch, no TensorFlow):
//   * crc32c (Castagnoli) + TF/LevelDB masking,
//   * TensorFlow TensorBundle-V2 checkpoints (SSTable ``.index`` + raw ``.data-XXXXX-of-YYYYY``),
//   * TFRecord / tf.Event summary files (``events.out.tfevents.*``),
//   * the CIFAR-10 binary-record reader.
// Replaces the TF C++ runtime pieces the reference exercises implicitly: SaveV2/RestoreV2 and the
// EventsWriter behind MonitoredTrainingSession (/root/reference/cifar10cnn.py:222) and the
// FixedLengthRecordReader/DecodeRaw input ops (cifar10cnn.py:54-70); SURVEY.md §2.B N1, N16.
#pragma once
#include <cstdint>
#include <string>
#include <vector>

namespace dmlc_rt {

// ---- crc32c ------------------------------------------------------------------------------------
uint32_t crc32c_extend(uint32_t crc, const uint8_t* data, size_t n);
inline uint32_t crc32c(const uint8_t* data, size_t n) { return crc32c_extend(0, data, n); }
inline uint32_t crc_mask(uint32_t crc) { return ((crc >> 15) | (crc << 17)) + 0xa282ead8u; }
inline uint32_t crc_unmask(uint32_t m) {
  const uint32_t rot = m - 0xa282ead8u;
  return (rot >> 17) | (rot << 15);
}

// ---- little-endian / varint coding -------------------------------------------------------------
void put_fixed32(std::string* dst, uint32_t v);
void put_fixed64(std::string* dst, uint64_t v);
void put_varint(std::string* dst, uint64_t v);
uint32_t get_fixed32(const uint8_t* p);
uint64_t get_fixed64(const uint8_t* p);
// Returns the pointer past the varint, or nullptr on malformed input.
const uint8_t* get_varint(const uint8_t* p, const uint8_t* end, uint64_t* v);

// ---- TensorBundle ------------------------------------------------------------------------------
// TF DataType enum values used by the bundle (tensorflow/core/framework/types.proto).
enum TfDType : int { DT_FLOAT = 1, DT_DOUBLE = 2, DT_INT32 = 3, DT_UINT8 = 4, DT_INT16 = 5, DT_INT8 = 6,
                     DT_INT64 = 9, DT_BOOL = 10, DT_BFLOAT16 = 14, DT_HALF = 19 };
int dtype_size(int dtype);

struct BundleEntry {
  std::string name;
  int dtype = 0;
  std::vector<int64_t> shape;
  int shard_id = 0;
  int64_t offset = 0;
  int64_t size = 0;
  uint32_t crc32c = 0;      // unmasked crc32c of the tensor bytes
};

// Serialisers (exposed for golden tests).
std::string encode_header(int num_shards);
std::string encode_entry(const BundleEntry& e);
bool decode_entry(const std::string& bytes, BundleEntry* e, std::string* err);

// LevelDB/TF table (SSTable) builder: keys must be added in strictly increasing byte order.
class TableBuilder {
 public:
  explicit TableBuilder(size_t block_size = 262144, int restart_interval = 16)
      : block_size_(block_size), restart_interval_(restart_interval) {}
  void add(const std::string& key, const std::string& value);
  std::string finish();   // whole file image

 private:
  struct Block {
    std::string buf;
    std::vector<uint32_t> restarts{0};
    int counter = 0;
    std::string last_key;
    bool empty() const { return buf.empty(); }
  };
  static void block_add(Block* b, int interval, const std::string& key, const std::string& value);
  static std::string block_finish(Block* b);
  void write_block(Block* b, uint64_t* off, uint64_t* size);
  void flush();

  size_t block_size_;
  int restart_interval_;
  std::string out_;
  Block data_, index_;
  bool pending_index_ = false;
  uint64_t pending_off_ = 0, pending_size_ = 0;
  std::string last_key_;
};

// Parses an SSTable image; fills (key, value) pairs in order.  Verifies every block checksum.
bool read_table(const std::string& image, std::vector<std::pair<std::string, std::string>>* kv,
                std::string* err);

// Writes <prefix>.index and <prefix>.data-00000-of-00001.  Entries are sorted by name; their
// tensor bytes are laid out in that order.  Returns "" on success, else an error message.
std::string write_bundle(const std::string& prefix, const std::vector<std::string>& names,
                         const std::vector<int>& dtypes, const std::vector<std::vector<int64_t>>& shapes,
                         const std::vector<std::string>& data);

// Reads a bundle (any number of shards).  Verifies the per-tensor crc32c.
std::string read_bundle(const std::string& prefix, std::vector<BundleEntry>* entries,
                        std::vector<std::string>* data);

// ---- TFRecord / events -------------------------------------------------------------------------
std::string tfrecord_frame(const std::string& payload);
std::string encode_event_file_version(double wall_time);
std::string encode_event_scalars(double wall_time, int64_t step, const std::vector<std::string>& tags,
                                 const std::vector<float>& values);

// ---- CIFAR-10 binary ---------------------------------------------------------------------------
// Parses 3073-byte records (label byte + 3x32x32 CHW) of every file, in order, into NHWC uint8
// images (out_images: n*3072 bytes) and int32 labels.  Multithreaded.  Returns "" or an error.
std::string read_cifar_files(const std::vector<std::string>& files, std::vector<uint8_t>* images,
                             std::vector<int32_t>* labels, int threads);

}  // namespace dmlc_rt
