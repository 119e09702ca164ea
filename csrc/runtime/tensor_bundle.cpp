// TensorFlow TensorBundle-V2 checkpoint format, written and read natively (no TF, no protobuf lib).
//
// What TF1's Saver (V2, sharded) produces for the reference's MonitoredTrainingSession
// (/root/reference/cifar10cnn.py:222):
//   <prefix>.index                  LevelDB-format table (SSTable), keys sorted bytewise:
//                                   ""        -> BundleHeaderProto {num_shards, endianness, version}
//                                   <tensor>  -> BundleEntryProto  {dtype, shape, shard_id, offset, size, crc32c}
//   <prefix>.data-%05d-of-%05d      the raw little-endian tensor bytes, concatenated.
// Table layout: data block(s) [entries with key prefix compression, restart array] + 5-byte trailer
// (compression type 0 + masked crc32c), an empty metaindex block, the index block (restart interval
// 1; separator keys shortened like LevelDB's BytewiseComparator), and the 48-byte footer ending in
// the magic 0xdb4775248b80fb57.  Protos are hand-encoded (proto3: default-valued scalars omitted).
#include "rt.h"

#include <algorithm>
#include <cstdio>
#include <cstring>
#include <fstream>
#include <map>
#include <numeric>
#include <sstream>

namespace dmlc_rt {

namespace {
constexpr uint64_t kTableMagic = 0xdb4775248b80fb57ull;
constexpr size_t kFooterSize = 48;  // 2 * BlockHandle::kMaxEncodedLength (20) + 8

void put_tag(std::string* d, int field, int wire) { put_varint(d, (uint64_t)((field << 3) | wire)); }
void put_len_field(std::string* d, int field, const std::string& payload) {
  put_tag(d, field, 2);
  put_varint(d, payload.size());
  d->append(payload);
}

// LevelDB BytewiseComparator::FindShortestSeparator / FindShortSuccessor
void shortest_separator(std::string* start, const std::string& limit) {
  const size_t n = std::min(start->size(), limit.size());
  size_t i = 0;
  while (i < n && (*start)[i] == limit[i]) ++i;
  if (i >= n) return;  // one is a prefix of the other
  const uint8_t b = (uint8_t)(*start)[i];
  if (b < 0xff && b + 1 < (uint8_t)limit[i]) {
    (*start)[i] = (char)(b + 1);
    start->resize(i + 1);
  }
}
void short_successor(std::string* key) {
  for (size_t i = 0; i < key->size(); ++i) {
    const uint8_t b = (uint8_t)(*key)[i];
    if (b != 0xff) {
      (*key)[i] = (char)(b + 1);
      key->resize(i + 1);
      return;
    }
  }
}

std::string encode_handle(uint64_t off, uint64_t size) {
  std::string s;
  put_varint(&s, off);
  put_varint(&s, size);
  return s;
}

bool read_file(const std::string& path, std::string* out) {
  std::ifstream f(path, std::ios::binary);
  if (!f) return false;
  std::ostringstream ss;
  ss << f.rdbuf();
  *out = ss.str();
  return true;
}

bool write_file_atomic(const std::string& path, const std::string& data) {
  const std::string tmp = path + ".tempstate";
  {
    std::ofstream f(tmp, std::ios::binary | std::ios::trunc);
    if (!f) return false;
    f.write(data.data(), (std::streamsize)data.size());
    if (!f) return false;
  }
  return std::rename(tmp.c_str(), path.c_str()) == 0;
}

std::string shard_name(const std::string& prefix, int shard, int num) {
  char b[64];
  std::snprintf(b, sizeof(b), ".data-%05d-of-%05d", shard, num);
  return prefix + b;
}

// parse one block's entries; appends to kv
bool parse_block(const uint8_t* p, size_t n, std::vector<std::pair<std::string, std::string>>* kv, std::string* err) {
  if (n < 4) { *err = "block too small"; return false; }
  const uint32_t nrest = get_fixed32(p + n - 4);
  if ((size_t)nrest * 4 + 4 > n) { *err = "bad restart count"; return false; }
  const uint8_t* end = p + n - 4 - 4 * (size_t)nrest;
  std::string key;
  while (p < end) {
    uint64_t shared, nonshared, vlen;
    p = get_varint(p, end, &shared);
    if (p) p = get_varint(p, end, &nonshared);
    if (p) p = get_varint(p, end, &vlen);
    if (!p || shared > key.size() || (uint64_t)(end - p) < nonshared + vlen) { *err = "corrupt block entry"; return false; }
    key.resize(shared);
    key.append((const char*)p, nonshared);
    p += nonshared;
    kv->emplace_back(key, std::string((const char*)p, vlen));
    p += vlen;
  }
  return true;
}

bool read_block(const std::string& img, uint64_t off, uint64_t size, std::vector<std::pair<std::string, std::string>>* kv,
                std::string* err) {
  if (off + size + 5 > img.size()) { *err = "block handle out of range"; return false; }
  const uint8_t* p = (const uint8_t*)img.data() + off;
  if (p[size] != 0) { *err = "compressed blocks are not supported"; return false; }
  const uint32_t want = crc_unmask(get_fixed32(p + size + 1));
  const uint32_t got = crc32c_extend(crc32c(p, size), p + size, 1);
  if (want != got) { *err = "block checksum mismatch"; return false; }
  return parse_block(p, size, kv, err);
}
}  // namespace

int dtype_size(int dt) {
  switch (dt) {
    case DT_FLOAT: case DT_INT32: return 4;
    case DT_DOUBLE: case DT_INT64: return 8;
    case DT_UINT8: case DT_INT8: case DT_BOOL: return 1;
    case DT_INT16: case DT_BFLOAT16: case DT_HALF: return 2;
    default: return 0;
  }
}

std::string encode_header(int num_shards) {
  std::string s, ver;
  if (num_shards) { put_tag(&s, 1, 0); put_varint(&s, (uint64_t)num_shards); }
  // endianness LITTLE = 0 (default, omitted); version {producer: 1}
  put_tag(&ver, 1, 0);
  put_varint(&ver, 1);
  put_len_field(&s, 3, ver);
  return s;
}

std::string encode_entry(const BundleEntry& e) {
  std::string s, shape;
  if (e.dtype) { put_tag(&s, 1, 0); put_varint(&s, (uint64_t)e.dtype); }
  for (int64_t d : e.shape) {
    std::string dim;
    if (d) { put_tag(&dim, 1, 0); put_varint(&dim, (uint64_t)d); }
    put_len_field(&shape, 2, dim);
  }
  put_len_field(&s, 2, shape);  // always present (a scalar has an empty TensorShapeProto)
  if (e.shard_id) { put_tag(&s, 3, 0); put_varint(&s, (uint64_t)e.shard_id); }
  if (e.offset) { put_tag(&s, 4, 0); put_varint(&s, (uint64_t)e.offset); }
  if (e.size) { put_tag(&s, 5, 0); put_varint(&s, (uint64_t)e.size); }
  put_tag(&s, 6, 5);
  put_fixed32(&s, crc_mask(e.crc32c));  // TF stores the MASKED crc32c of the tensor bytes
  return s;
}

namespace {
// generic proto field walker
template <class F>
bool walk_proto(const uint8_t* p, const uint8_t* end, F&& on_field) {
  while (p < end) {
    uint64_t tag;
    p = get_varint(p, end, &tag);
    if (!p) return false;
    const int field = (int)(tag >> 3), wire = (int)(tag & 7);
    uint64_t v = 0;
    const uint8_t* sub = nullptr;
    size_t sublen = 0;
    if (wire == 0) {
      p = get_varint(p, end, &v);
      if (!p) return false;
    } else if (wire == 1) {
      if (end - p < 8) return false;
      v = get_fixed64(p);
      p += 8;
    } else if (wire == 5) {
      if (end - p < 4) return false;
      v = get_fixed32(p);
      p += 4;
    } else if (wire == 2) {
      uint64_t len;
      p = get_varint(p, end, &len);
      if (!p || (uint64_t)(end - p) < len) return false;
      sub = p;
      sublen = (size_t)len;
      p += len;
    } else {
      return false;
    }
    if (!on_field(field, wire, v, sub, sublen)) return false;
  }
  return true;
}
}  // namespace

bool decode_entry(const std::string& bytes, BundleEntry* e, std::string* err) {
  const uint8_t* p = (const uint8_t*)bytes.data();
  bool has_slices = false;
  const bool ok = walk_proto(p, p + bytes.size(), [&](int f, int w, uint64_t v, const uint8_t* sub, size_t n) {
    if (f == 1 && w == 0) e->dtype = (int)v;
    else if (f == 2 && w == 2) {
      e->shape.clear();
      return walk_proto(sub, sub + n, [&](int f2, int w2, uint64_t, const uint8_t* s2, size_t n2) {
        if (f2 == 2 && w2 == 2) {
          int64_t size = 0;
          if (!walk_proto(s2, s2 + n2, [&](int f3, int w3, uint64_t v3, const uint8_t*, size_t) {
                if (f3 == 1 && w3 == 0) size = (int64_t)v3;
                return true;
              }))
            return false;
          e->shape.push_back(size);
        }
        return true;
      });
    } else if (f == 3 && w == 0) e->shard_id = (int)v;
    else if (f == 4 && w == 0) e->offset = (int64_t)v;
    else if (f == 5 && w == 0) e->size = (int64_t)v;
    else if (f == 6 && w == 5) e->crc32c = crc_unmask((uint32_t)v);
    else if (f == 7) has_slices = true;
    return true;
  });
  if (!ok) { *err = "corrupt BundleEntryProto for '" + e->name + "'"; return false; }
  if (has_slices) { *err = "partitioned (sliced) variables are not supported: '" + e->name + "'"; return false; }
  return true;
}

// ---- table builder ---------------------------------------------------------------------------
void TableBuilder::block_add(Block* b, int interval, const std::string& key, const std::string& value) {
  size_t shared = 0;
  if (b->counter < interval) {
    const size_t n = std::min(b->last_key.size(), key.size());
    while (shared < n && b->last_key[shared] == key[shared]) ++shared;
  } else {
    b->restarts.push_back((uint32_t)b->buf.size());
    b->counter = 0;
  }
  put_varint(&b->buf, shared);
  put_varint(&b->buf, key.size() - shared);
  put_varint(&b->buf, value.size());
  b->buf.append(key, shared, std::string::npos);
  b->buf.append(value);
  b->last_key = key;
  ++b->counter;
}

std::string TableBuilder::block_finish(Block* b) {
  std::string out = b->buf;
  for (uint32_t r : b->restarts) put_fixed32(&out, r);
  put_fixed32(&out, (uint32_t)b->restarts.size());
  *b = Block();
  return out;
}

void TableBuilder::write_block(Block* b, uint64_t* off, uint64_t* size) {
  const std::string contents = block_finish(b);
  *off = out_.size();
  *size = contents.size();
  out_.append(contents);
  const char type = 0;
  out_.push_back(type);
  const uint32_t crc = crc32c_extend(crc32c((const uint8_t*)contents.data(), contents.size()), (const uint8_t*)&type, 1);
  put_fixed32(&out_, crc_mask(crc));
}

void TableBuilder::flush() {
  if (data_.empty()) return;
  write_block(&data_, &pending_off_, &pending_size_);
  pending_index_ = true;
}

void TableBuilder::add(const std::string& key, const std::string& value) {
  if (pending_index_) {
    std::string sep = last_key_;
    shortest_separator(&sep, key);
    block_add(&index_, 1, sep, encode_handle(pending_off_, pending_size_));
    pending_index_ = false;
  }
  block_add(&data_, restart_interval_, key, value);
  last_key_ = key;
  if (data_.buf.size() + 4 * data_.restarts.size() + 4 >= block_size_) flush();
}

std::string TableBuilder::finish() {
  flush();
  Block meta;
  uint64_t meta_off, meta_size, idx_off, idx_size;
  write_block(&meta, &meta_off, &meta_size);
  if (pending_index_) {
    std::string succ = last_key_;
    short_successor(&succ);
    block_add(&index_, 1, succ, encode_handle(pending_off_, pending_size_));
    pending_index_ = false;
  }
  write_block(&index_, &idx_off, &idx_size);
  std::string footer = encode_handle(meta_off, meta_size) + encode_handle(idx_off, idx_size);
  footer.resize(kFooterSize - 8, '\0');
  put_fixed64(&footer, kTableMagic);
  out_.append(footer);
  return out_;
}

bool read_table(const std::string& img, std::vector<std::pair<std::string, std::string>>* kv, std::string* err) {
  if (img.size() < kFooterSize) { *err = "file too small for a table footer"; return false; }
  const uint8_t* f = (const uint8_t*)img.data() + img.size() - kFooterSize;
  if (get_fixed64(f + kFooterSize - 8) != kTableMagic) { *err = "bad table magic"; return false; }
  uint64_t mo, ms, io, is;
  const uint8_t* fe = f + kFooterSize - 8;
  const uint8_t* p = get_varint(f, fe, &mo);
  if (p) p = get_varint(p, fe, &ms);
  if (p) p = get_varint(p, fe, &io);
  if (p) p = get_varint(p, fe, &is);
  if (!p) { *err = "corrupt footer"; return false; }
  std::vector<std::pair<std::string, std::string>> index;
  if (!read_block(img, io, is, &index, err)) return false;
  for (auto& e : index) {
    uint64_t off, size;
    const uint8_t* h = (const uint8_t*)e.second.data();
    const uint8_t* he = h + e.second.size();
    h = get_varint(h, he, &off);
    if (h) h = get_varint(h, he, &size);
    if (!h) { *err = "corrupt block handle"; return false; }
    if (!read_block(img, off, size, kv, err)) return false;
  }
  return true;
}

std::string write_bundle(const std::string& prefix, const std::vector<std::string>& names, const std::vector<int>& dtypes,
                         const std::vector<std::vector<int64_t>>& shapes, const std::vector<std::string>& data) {
  const size_t n = names.size();
  if (dtypes.size() != n || shapes.size() != n || data.size() != n) return "write_bundle: list lengths differ";
  std::vector<size_t> order(n);
  std::iota(order.begin(), order.end(), 0);
  std::sort(order.begin(), order.end(), [&](size_t a, size_t b) { return names[a] < names[b]; });
  for (size_t i = 1; i < n; ++i)
    if (names[order[i]] == names[order[i - 1]]) return "duplicate tensor name '" + names[order[i]] + "'";
  std::string blob;
  TableBuilder tb;
  tb.add("", encode_header(1));
  for (size_t oi : order) {
    if (names[oi].empty()) return "empty tensor name";
    const int es = dtype_size(dtypes[oi]);
    if (!es) return "unsupported dtype for '" + names[oi] + "'";
    int64_t numel = 1;
    for (int64_t d : shapes[oi]) numel *= d;
    if ((int64_t)data[oi].size() != numel * es) return "byte size mismatch for '" + names[oi] + "'";
    BundleEntry e;
    e.name = names[oi];
    e.dtype = dtypes[oi];
    e.shape = shapes[oi];
    e.offset = (int64_t)blob.size();
    e.size = (int64_t)data[oi].size();
    e.crc32c = crc32c((const uint8_t*)data[oi].data(), data[oi].size());
    blob.append(data[oi]);
    tb.add(e.name, encode_entry(e));
  }
  if (!write_file_atomic(shard_name(prefix, 0, 1), blob)) return "cannot write " + shard_name(prefix, 0, 1);
  // the index goes last: its presence marks a complete checkpoint
  if (!write_file_atomic(prefix + ".index", tb.finish())) return "cannot write " + prefix + ".index";
  return "";
}

std::string read_bundle(const std::string& prefix, std::vector<BundleEntry>* entries, std::vector<std::string>* data) {
  std::string img, err;
  if (!read_file(prefix + ".index", &img)) return "cannot read " + prefix + ".index";
  std::vector<std::pair<std::string, std::string>> kv;
  if (!read_table(img, &kv, &err)) return prefix + ".index: " + err;
  if (kv.empty() || !kv[0].first.empty()) return "missing bundle header entry";
  int num_shards = 1;
  {
    const uint8_t* p = (const uint8_t*)kv[0].second.data();
    int endian = 0;
    walk_proto(p, p + kv[0].second.size(), [&](int f, int w, uint64_t v, const uint8_t*, size_t) {
      if (f == 1 && w == 0) num_shards = (int)v;
      if (f == 2 && w == 0) endian = (int)v;
      return true;
    });
    if (endian != 0) return "big-endian bundles are not supported";
  }
  std::map<int, std::string> shards;
  for (size_t i = 1; i < kv.size(); ++i) {
    BundleEntry e;
    e.name = kv[i].first;
    if (!decode_entry(kv[i].second, &e, &err)) return err;
    if (e.shard_id < 0 || e.shard_id >= num_shards) return "bad shard id for '" + e.name + "'";
    auto it = shards.find(e.shard_id);
    if (it == shards.end()) {
      std::string blob;
      if (!read_file(shard_name(prefix, e.shard_id, num_shards), &blob))
        return "cannot read " + shard_name(prefix, e.shard_id, num_shards);
      it = shards.emplace(e.shard_id, std::move(blob)).first;
    }
    if (e.offset < 0 || e.size < 0 || (size_t)(e.offset + e.size) > it->second.size())
      return "tensor '" + e.name + "' out of range of its data file";
    std::string bytes = it->second.substr((size_t)e.offset, (size_t)e.size);
    if (crc32c((const uint8_t*)bytes.data(), bytes.size()) != e.crc32c) return "crc32c mismatch for '" + e.name + "'";
    entries->push_back(e);
    data->push_back(std::move(bytes));
  }
  return "";
}

}  // namespace dmlc_rt
