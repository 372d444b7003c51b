// TensorFlow checkpoint V2 ("tensor bundle") writer/reader, natively.
//
// The reference saves with `tf.train.Saver()` (model_export.py:53) and the
// BASELINE north star requires the TF checkpoint format to stay compatible.
// A V2 checkpoint `prefix` is:
//   prefix.index                 leveldb-format SSTable, key "" -> BundleHeaderProto,
//                                key <tensor name> -> BundleEntryProto (sorted keys)
//   prefix.data-0000k-of-0000N   raw little-endian tensor bytes
// SSTable layout: data blocks (prefix-compressed entries + restart array),
// each followed by a 5-byte trailer {type=0 (uncompressed), masked crc32c};
// an empty metaindex block; an index block (restart interval 1) mapping a
// key >= every key of a data block to its BlockHandle; a 48-byte footer
// {metaindex handle, index handle, zero pad to 40 B, magic 0xdb4775248b80fb57}.
// Proto fields (proto3, zero scalars omitted):
//   BundleHeaderProto{num_shards=1, endianness=2, version=3{producer=1,min_consumer=2}}
//   BundleEntryProto {dtype=1, shape=2{dim=2{size=1,name=2}}, shard_id=3, offset=4,
//                     size=5, crc32c=6 (fixed32, masked crc of the bytes), slices=7}
//   TensorSliceProto {extent=1{start=1, length=2 (oneof: absent = full extent)}}
// Partitioned variables (TF Saver + SaveSliceInfo, [TF-semantics]): the full
// tensor's key carries dtype, full shape and one TensorSliceProto per saved
// slice, and no data; each slice's bytes live under the key
// EncodeTensorNameSlice(name, slice) = OrderedCode NumIncreasing(0), String(name),
// NumIncreasing(dims), then per dim SignedNumIncreasing(start),
// SignedNumIncreasing(length) (length -1 = full).  Like SaveV2, every slice of
// a partitioned variable goes through this path (even a single partition).
// Shard indexes merge the slice lists of a full key written by several shards.
#include <torch/extension.h>

#include <algorithm>
#include <cstdio>
#include <map>
#include <string>
#include <vector>

#include "crc32c.h"
#include "wire.h"

namespace dtf {
namespace bundle {

constexpr uint64_t kTableMagic = 0xdb4775248b80fb57ull;
constexpr size_t kBlockSize = 256 * 1024;
constexpr int kRestartInterval = 16;

struct Handle {
  uint64_t offset = 0, size = 0;
  void encode(std::string& s) const {
    wire::put_varint(s, offset);
    wire::put_varint(s, size);
  }
};

class BlockBuilder {
 public:
  explicit BlockBuilder(int restart_interval) : interval_(restart_interval) { restarts_.push_back(0); }
  void add(const std::string& key, const std::string& value) {
    size_t shared = 0;
    if (counter_ < interval_) {
      size_t m = std::min(last_.size(), key.size());
      while (shared < m && last_[shared] == key[shared]) ++shared;
    } else {
      restarts_.push_back((uint32_t)buf_.size());
      counter_ = 0;
    }
    wire::put_varint(buf_, shared);
    wire::put_varint(buf_, key.size() - shared);
    wire::put_varint(buf_, value.size());
    buf_.append(key.data() + shared, key.size() - shared);
    buf_.append(value);
    last_ = key;
    ++counter_;
    ++n_;
  }
  std::string finish() {
    std::string out = buf_;
    for (uint32_t r : restarts_) wire::put_fixed32(out, r);
    wire::put_fixed32(out, (uint32_t)restarts_.size());
    return out;
  }
  size_t estimate() const { return buf_.size() + restarts_.size() * 4 + 4; }
  bool empty() const { return n_ == 0; }
  void reset() {
    buf_.clear();
    restarts_.assign(1, 0);
    counter_ = 0;
    n_ = 0;
    last_.clear();
  }

 private:
  int interval_;
  std::string buf_, last_;
  std::vector<uint32_t> restarts_;
  int counter_ = 0;
  size_t n_ = 0;
};

class TableWriter {
 public:
  explicit TableWriter(const std::string& path) : data_(kRestartInterval), index_(1) {
    f_ = fopen(path.c_str(), "wb");
    if (!f_) throw std::runtime_error("cannot create " + path);
  }
  ~TableWriter() {
    if (f_) fclose(f_);
  }
  void add(const std::string& key, const std::string& value) {
    if (pending_index_) {
      std::string h;
      pending_handle_.encode(h);
      index_.add(last_key_, h);
      pending_index_ = false;
    }
    data_.add(key, value);
    last_key_ = key;
    if (data_.estimate() >= kBlockSize) flush_data();
  }
  void finish() {
    flush_data();
    if (pending_index_) {
      std::string h;
      pending_handle_.encode(h);
      index_.add(last_key_, h);
      pending_index_ = false;
    }
    BlockBuilder meta(kRestartInterval);
    Handle mh = write_block(meta.finish());
    Handle ih = write_block(index_.finish());
    std::string footer;
    mh.encode(footer);
    ih.encode(footer);
    footer.resize(40, '\0');
    wire::put_fixed64(footer, kTableMagic);
    fwrite(footer.data(), 1, footer.size(), f_);
    fclose(f_);
    f_ = nullptr;
  }

 private:
  void flush_data() {
    if (data_.empty()) return;
    pending_handle_ = write_block(data_.finish());
    pending_index_ = true;
    data_.reset();
  }
  Handle write_block(const std::string& contents) {
    Handle h;
    h.offset = off_;
    h.size = contents.size();
    char type = 0;
    uint32_t crc = crc32c_extend(crc32c(contents.data(), contents.size()), &type, 1);
    std::string trailer(1, type);
    wire::put_fixed32(trailer, crc32c_mask(crc));
    fwrite(contents.data(), 1, contents.size(), f_);
    fwrite(trailer.data(), 1, trailer.size(), f_);
    off_ += contents.size() + trailer.size();
    return h;
  }
  FILE* f_ = nullptr;
  BlockBuilder data_, index_;
  std::string last_key_;
  Handle pending_handle_;
  bool pending_index_ = false;
  uint64_t off_ = 0;
};

static std::string read_file(const std::string& path) {
  FILE* f = fopen(path.c_str(), "rb");
  if (!f) throw std::runtime_error("cannot open " + path);
  fseek(f, 0, SEEK_END);
  long n = ftell(f);
  fseek(f, 0, SEEK_SET);
  std::string s(n, '\0');
  if (n > 0 && fread(&s[0], 1, n, f) != (size_t)n) {
    fclose(f);
    throw std::runtime_error("short read " + path);
  }
  fclose(f);
  return s;
}

static Handle decode_handle(wire::Reader& r) {
  Handle h;
  h.offset = r.varint();
  h.size = r.varint();
  return h;
}

static std::string block_at(const std::string& file, const Handle& h, bool verify) {
  if (h.offset + h.size + 5 > file.size()) throw std::runtime_error("block out of range");
  std::string contents = file.substr(h.offset, h.size);
  if (verify) {
    const char type = file[h.offset + h.size];
    uint32_t stored;
    memcpy(&stored, file.data() + h.offset + h.size + 1, 4);
    uint32_t crc = crc32c_extend(crc32c(contents.data(), contents.size()), &type, 1);
    if (crc32c_mask(crc) != stored) throw std::runtime_error("SSTable block checksum mismatch");
    if (type != 0) throw std::runtime_error("compressed SSTable blocks are not supported");
  }
  return contents;
}

static void parse_block(const std::string& b, std::vector<std::pair<std::string, std::string>>& out) {
  if (b.size() < 4) throw std::runtime_error("bad block");
  uint32_t nrest;
  memcpy(&nrest, b.data() + b.size() - 4, 4);
  size_t limit = b.size() - 4 - 4 * (size_t)nrest;
  wire::Reader r(b.data(), limit);
  std::string key;
  while (!r.done()) {
    uint64_t shared = r.varint(), nonshared = r.varint(), vlen = r.varint();
    if (shared > key.size() || (uint64_t)(r.end - r.p) < nonshared + vlen) throw std::runtime_error("bad entry");
    key.resize(shared);
    key.append(reinterpret_cast<const char*>(r.p), nonshared);
    r.p += nonshared;
    std::string val(reinterpret_cast<const char*>(r.p), vlen);
    r.p += vlen;
    out.emplace_back(key, val);
  }
}

// All (key, value) pairs of an SSTable, in order.
static std::vector<std::pair<std::string, std::string>> read_table(const std::string& path, bool verify) {
  std::string file = read_file(path);
  if (file.size() < 48) throw std::runtime_error("table too small: " + path);
  uint64_t magic;
  memcpy(&magic, file.data() + file.size() - 8, 8);
  if (magic != kTableMagic) throw std::runtime_error("bad table magic: " + path);
  wire::Reader fr(file.data() + file.size() - 48, 40);
  Handle mh = decode_handle(fr);
  Handle ih = decode_handle(fr);
  (void)mh;
  std::vector<std::pair<std::string, std::string>> idx, out;
  parse_block(block_at(file, ih, verify), idx);
  for (auto& kv : idx) {
    wire::Reader hr(kv.second.data(), kv.second.size());
    Handle h = decode_handle(hr);
    parse_block(block_at(file, h, verify), out);
  }
  return out;
}

// ---- OrderedCode (tensorflow/core/lib/strings/ordered_code) subset used by slice keys
static void oc_num_increasing(std::string& d, uint64_t v) {
  unsigned char buf[9];
  int len = 0;
  while (v > 0) {
    ++len;
    buf[9 - len] = (unsigned char)(v & 0xff);
    v >>= 8;
  }
  buf[9 - len - 1] = (unsigned char)len;
  d.append(reinterpret_cast<const char*>(buf + 9 - len - 1), len + 1);
}
static void oc_string(std::string& d, const std::string& s) {
  for (char c : s) {
    if (c == '\x00') d.append("\x00\xff", 2);
    else if (c == '\xff') d.append("\xff\x00", 2);
    else d.push_back(c);
  }
  d.append("\x00\x01", 2);
}
static void oc_signed_num_increasing(std::string& d, int64_t val) {
  static const unsigned char kHeader[11][2] = {{0, 0},       {0x80, 0}, {0xc0, 0}, {0xe0, 0},
                                               {0xf0, 0},    {0xf8, 0}, {0xfc, 0}, {0xfe, 0},
                                               {0xff, 0},    {0xff, 0x80}, {0xff, 0xc0}};
  const uint64_t x = val < 0 ? ~(uint64_t)val : (uint64_t)val;
  if (x < 64) {
    d.push_back((char)(kHeader[1][0] ^ (unsigned char)val));
    return;
  }
  // significant bits after the sign -> encoded length (7 payload bits per byte)
  int bits = 64 - __builtin_clzll(x);
  int len = (bits + 1 + 6) / 7;   // bits 7..13 -> 2, 14..20 -> 3, ...
  if (len > 10) len = 10;
  unsigned char buf[10];
  const unsigned char sign = val < 0 ? 0xff : 0x00;
  buf[0] = buf[1] = sign;
  for (int i = 0; i < 8; ++i) buf[2 + i] = (unsigned char)((uint64_t)val >> (56 - 8 * i));
  unsigned char* b = buf + 10 - len;
  b[0] ^= kHeader[len][0];
  b[1] ^= kHeader[len][1];
  d.append(reinterpret_cast<const char*>(b), len);
}
using Extents = std::vector<std::pair<int64_t, int64_t>>;   // (start, length); length -1 = full
static std::string encode_slice_key(const std::string& name, const Extents& ext) {
  std::string k;
  oc_num_increasing(k, 0);
  oc_string(k, name);
  oc_num_increasing(k, ext.size());
  for (auto& e : ext) {
    oc_signed_num_increasing(k, e.second < 0 ? 0 : e.first);
    oc_signed_num_increasing(k, e.second);
  }
  return k;
}
static std::string encode_slice_proto(const Extents& ext) {
  std::string sp;
  for (auto& e : ext) {
    std::string x;
    if (e.second >= 0) {
      if (e.first) wire::put_int(x, 1, e.first);
      wire::put_int(x, 2, e.second);   // oneof member: serialized even when 0
    }
    wire::put_bytes(sp, 1, x);
  }
  return sp;
}
static Extents decode_slice_proto(const std::string& sp) {
  Extents out;
  wire::Reader r(sp.data(), sp.size());
  int f, wt;
  while (r.next(f, wt)) {
    if (f == 1 && wt == wire::LEN) {
      std::string x = r.bytes();
      wire::Reader xr(x.data(), x.size());
      int64_t start = 0, len = -1;
      int f2, w2;
      while (xr.next(f2, w2)) {
        if (f2 == 1 && w2 == wire::VARINT) start = (int64_t)xr.varint();
        else if (f2 == 2 && w2 == wire::VARINT) len = (int64_t)xr.varint();
        else xr.skip(w2);
      }
      out.emplace_back(start, len);
    } else r.skip(wt);
  }
  return out;
}

struct Entry {
  int dtype = 0;
  std::vector<int64_t> shape;
  int shard_id = 0;
  int64_t offset = 0, size = 0;
  uint32_t crc = 0;
  std::string slices_raw;  // serialized TensorSliceProto(s), kept opaque
};

static std::string encode_entry(const Entry& e) {
  std::string s, shp;
  if (e.dtype) wire::put_uint(s, 1, (uint64_t)e.dtype);
  for (int64_t d : e.shape) {
    std::string dim;
    if (d) wire::put_int(dim, 1, d);
    wire::put_bytes(shp, 2, dim);
  }
  wire::put_bytes(s, 2, shp);
  if (e.shard_id) wire::put_int(s, 3, e.shard_id);
  if (e.offset) wire::put_int(s, 4, e.offset);
  if (e.size) wire::put_int(s, 5, e.size);
  if (e.crc) wire::put_fixed32_field(s, 6, e.crc);
  s.append(e.slices_raw);
  return s;
}

static Entry decode_entry(const std::string& v) {
  Entry e;
  wire::Reader r(v.data(), v.size());
  int f, wt;
  while (r.next(f, wt)) {
    if (f == 1 && wt == wire::VARINT) e.dtype = (int)r.varint();
    else if (f == 2 && wt == wire::LEN) {
      std::string shp = r.bytes();
      wire::Reader sr(shp.data(), shp.size());
      int f2, w2;
      while (sr.next(f2, w2)) {
        if (f2 == 2 && w2 == wire::LEN) {
          std::string dim = sr.bytes();
          wire::Reader dr(dim.data(), dim.size());
          int f3, w3;
          int64_t size = 0;
          while (dr.next(f3, w3)) {
            if (f3 == 1 && w3 == wire::VARINT) size = (int64_t)dr.varint();
            else dr.skip(w3);
          }
          e.shape.push_back(size);
        } else sr.skip(w2);
      }
    } else if (f == 3 && wt == wire::VARINT) e.shard_id = (int)r.varint();
    else if (f == 4 && wt == wire::VARINT) e.offset = (int64_t)r.varint();
    else if (f == 5 && wt == wire::VARINT) e.size = (int64_t)r.varint();
    else if (f == 6 && wt == wire::FIXED32) e.crc = r.fixed32();
    else if (f == 7 && wt == wire::LEN) {
      std::string sl = r.bytes();
      wire::put_bytes(e.slices_raw, 7, sl);
    } else r.skip(wt);
  }
  return e;
}

static std::string encode_header(int num_shards) {
  std::string h, ver;
  if (num_shards) wire::put_int(h, 1, num_shards);
  // endianness LITTLE = 0 -> omitted
  wire::put_int(ver, 1, 1);  // producer = kTensorBundleVersion
  wire::put_bytes(h, 3, ver);
  return h;
}

static std::string data_path(const std::string& prefix, int shard, int num_shards) {
  char buf[64];
  snprintf(buf, sizeof(buf), ".data-%05d-of-%05d", shard, num_shards);
  return prefix + buf;
}

static size_t dtype_size(int dt) {
  switch (dt) {
    case 1: return 4;   // DT_FLOAT
    case 2: return 8;   // DT_DOUBLE
    case 3: return 4;   // DT_INT32
    case 4: return 1;   // DT_UINT8
    case 5: return 2;   // DT_INT16
    case 6: return 1;   // DT_INT8
    case 9: return 8;   // DT_INT64
    case 10: return 1;  // DT_BOOL
    case 14: return 2;  // DT_BFLOAT16
    case 17: return 2;  // DT_UINT16
    case 19: return 2;  // DT_HALF
    case 22: return 4;  // DT_UINT32
    case 23: return 8;  // DT_UINT64
    default: return 0;
  }
}

// One shard's writer. With num_shards == 1 it also writes prefix.index.
// With num_shards > 1 each shard writes `prefix.index.shard-k` and the chief
// calls merge_shard_indexes().
class Writer {
 public:
  Writer(const std::string& prefix, int shard_id, int num_shards)
      : prefix_(prefix), shard_(shard_id), nshards_(num_shards) {
    f_ = fopen(data_path(prefix, shard_id, num_shards).c_str(), "wb");
    if (!f_) throw std::runtime_error("cannot create data file for " + prefix);
  }
  ~Writer() {
    if (f_) fclose(f_);
  }
  void add(const std::string& name, int dtype, std::vector<int64_t> shape, py::buffer buf) {
    if (name.empty()) throw std::runtime_error("empty tensor name");
    if (entries_.count(name)) throw std::runtime_error("duplicate tensor " + name);
    py::buffer_info info = buf.request();
    const size_t nbytes = (size_t)info.size * info.itemsize;
    int64_t numel = 1;
    for (auto d : shape) numel *= d;
    const size_t es = dtype_size(dtype);
    if (es && (size_t)numel * es != nbytes)
      throw std::runtime_error("byte size mismatch for " + name);
    Entry e;
    e.dtype = dtype;
    e.shape = shape;
    e.shard_id = shard_;
    e.offset = off_;
    e.size = (int64_t)nbytes;
    {
      py::gil_scoped_release nogil;
      e.crc = crc32c_mask(crc32c(info.ptr, nbytes));
      if (nbytes && fwrite(info.ptr, 1, nbytes, f_) != nbytes) throw std::runtime_error("write failed");
    }
    off_ += nbytes;
    entries_[name] = e;
  }
  // One slice of a partitioned variable: data under the slice key, the slice
  // recorded in the full tensor's entry (dtype, full shape, slices; no data).
  void add_slice(const std::string& full_name, int dtype, std::vector<int64_t> full_shape, Extents ext,
                 py::buffer buf) {
    if (full_name.empty()) throw std::runtime_error("empty tensor name");
    if (ext.size() != full_shape.size()) throw std::runtime_error("slice rank != tensor rank for " + full_name);
    std::vector<int64_t> sshape;
    for (size_t d = 0; d < ext.size(); ++d) {
      const int64_t len = ext[d].second < 0 ? full_shape[d] : ext[d].second;
      const int64_t st = ext[d].second < 0 ? 0 : ext[d].first;
      if (st < 0 || len < 0 || st + len > full_shape[d]) throw std::runtime_error("slice out of range: " + full_name);
      sshape.push_back(len);
    }
    Entry& fe = entries_[full_name];
    if (fe.size != 0 || (fe.dtype && fe.dtype != dtype) || (!fe.shape.empty() && fe.shape != full_shape))
      throw std::runtime_error("conflicting entries for sliced tensor " + full_name);
    fe.dtype = dtype;
    fe.shape = full_shape;
    fe.shard_id = 0;
    wire::put_bytes(fe.slices_raw, 7, encode_slice_proto(ext));
    add(encode_slice_key(full_name, ext), dtype, sshape, buf);
  }
  void finish() {
    if (f_) {
      fflush(f_);
      fclose(f_);
      f_ = nullptr;
    }
    std::string ipath = nshards_ == 1 ? prefix_ + ".index" : prefix_ + ".index.shard-" + std::to_string(shard_);
    TableWriter t(ipath);
    t.add("", encode_header(nshards_));
    for (auto& kv : entries_) t.add(kv.first, encode_entry(kv.second));  // std::map: sorted
    t.finish();
  }

 private:
  std::string prefix_;
  int shard_, nshards_;
  FILE* f_ = nullptr;
  uint64_t off_ = 0;
  std::map<std::string, Entry> entries_;
};

void merge_shard_indexes(const std::string& prefix, int num_shards, bool remove_parts) {
  std::map<std::string, std::string> all;
  for (int k = 0; k < num_shards; ++k) {
    std::string p = prefix + ".index.shard-" + std::to_string(k);
    for (auto& kv : read_table(p, true)) {
      if (kv.first.empty()) continue;
      auto it = all.find(kv.first);
      if (it == all.end()) {
        all[kv.first] = kv.second;
        continue;
      }
      // the same sliced tensor from several shards: concatenate the slice lists
      Entry a = decode_entry(it->second), b = decode_entry(kv.second);
      if (a.slices_raw.empty() || b.slices_raw.empty() || a.size || b.size || a.dtype != b.dtype || a.shape != b.shape)
        throw std::runtime_error("tensor in two shards: " + kv.first);
      a.slices_raw += b.slices_raw;
      it->second = encode_entry(a);
    }
    if (remove_parts) remove(p.c_str());
  }
  TableWriter t(prefix + ".index");
  t.add("", encode_header(num_shards));
  for (auto& kv : all) t.add(kv.first, kv.second);
  t.finish();
}

py::dict read_index(const std::string& prefix) {
  py::dict d;
  for (auto& kv : read_table(prefix + ".index", true)) {
    if (kv.first.empty()) {
      wire::Reader r(kv.second.data(), kv.second.size());
      int f, wt, ns = 1;
      while (r.next(f, wt)) {
        if (f == 1 && wt == wire::VARINT) ns = (int)r.varint();
        else r.skip(wt);
      }
      d[py::str("")] = py::dict(py::arg("num_shards") = ns);
      continue;
    }
    if (kv.first[0] == '\x00') continue;   // a slice's data entry (EncodeTensorNameSlice key)
    Entry e = decode_entry(kv.second);
    py::list slices;
    if (!e.slices_raw.empty()) {
      wire::Reader r(e.slices_raw.data(), e.slices_raw.size());
      int f, wt;
      while (r.next(f, wt)) {
        if (f == 7 && wt == wire::LEN) {
          py::list ext;
          for (auto& x : decode_slice_proto(r.bytes())) ext.append(py::make_tuple(x.first, x.second));
          slices.append(ext);
        } else r.skip(wt);
      }
    }
    d[py::str(kv.first)] = py::dict(py::arg("dtype") = e.dtype, py::arg("shape") = e.shape,
                                    py::arg("shard_id") = e.shard_id, py::arg("offset") = e.offset,
                                    py::arg("size") = e.size, py::arg("crc32c") = e.crc,
                                    py::arg("has_slices") = !e.slices_raw.empty(), py::arg("slices") = slices);
  }
  return d;
}

py::bytes read_tensor(const std::string& prefix, const std::string& name, bool verify) {
  int nshards = 1;
  Entry found;
  bool ok = false;
  for (auto& kv : read_table(prefix + ".index", true)) {
    if (kv.first.empty()) {
      wire::Reader r(kv.second.data(), kv.second.size());
      int f, wt;
      while (r.next(f, wt)) {
        if (f == 1 && wt == wire::VARINT) nshards = (int)r.varint();
        else r.skip(wt);
      }
    } else if (kv.first == name) {
      found = decode_entry(kv.second);
      ok = true;
    }
  }
  if (!ok) throw std::runtime_error("tensor not found in checkpoint: " + name);
  std::string path = data_path(prefix, found.shard_id, nshards);
  FILE* f = fopen(path.c_str(), "rb");
  if (!f) throw std::runtime_error("cannot open " + path);
  std::string buf(found.size, '\0');
  fseek(f, found.offset, SEEK_SET);
  size_t n = found.size ? fread(&buf[0], 1, found.size, f) : 0;
  fclose(f);
  if ((int64_t)n != found.size) throw std::runtime_error("short read of " + name);
  if (verify && crc32c_mask(crc32c(buf.data(), buf.size())) != found.crc)
    throw std::runtime_error("checksum mismatch for tensor " + name);
  return py::bytes(buf);
}

}  // namespace bundle

void init_bundle(py::module& m) {
  using namespace bundle;
  py::class_<Writer>(m, "BundleWriter")
      .def(py::init<const std::string&, int, int>(), py::arg("prefix"), py::arg("shard_id") = 0,
           py::arg("num_shards") = 1)
      .def("add", &Writer::add)
      .def("add_slice", &Writer::add_slice)
      .def("finish", &Writer::finish);
  m.def("bundle_merge_shard_indexes", &merge_shard_indexes, py::arg("prefix"), py::arg("num_shards"),
        py::arg("remove_parts") = true);
  m.def("bundle_read_index", &read_index);
  m.def("bundle_slice_key", [](const std::string& name, Extents ext) { return py::bytes(encode_slice_key(name, ext)); });
  m.def("bundle_read_slice", [](const std::string& prefix, const std::string& name, Extents ext, bool verify) {
    return read_tensor(prefix, encode_slice_key(name, ext), verify);
  }, py::arg("prefix"), py::arg("name"), py::arg("extents"), py::arg("verify") = true);
  m.def("bundle_read_tensor", &read_tensor, py::arg("prefix"), py::arg("name"), py::arg("verify") = true);
  m.def("sstable_read", [](const std::string& path) {
    py::list out;
    for (auto& kv : read_table(path, true)) out.append(py::make_tuple(py::bytes(kv.first), py::bytes(kv.second)));
    return out;
  });
  m.def("sstable_write", [](const std::string& path, std::vector<std::pair<std::string, std::string>> kvs) {
    std::sort(kvs.begin(), kvs.end());
    TableWriter t(path);
    for (auto& kv : kvs) t.add(kv.first, kv.second);
    t.finish();
  });
}

}  // namespace dtf
