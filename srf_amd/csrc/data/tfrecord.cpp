// TF-free TFRecord reader/writer and tf.train.Example codec for the speech
// records of the SRF input pipeline (include/srf_data.h).
//
// Replaces, without TensorFlow:
//   * tf.data.TFRecordDataset framing + CRC checks (load_speech_data.py:43-46);
//   * tf.io.parse_single_example with the VarLen/FixedLen spec of
//     load_speech_data.py:52-85 (input_speech float32, target_label int64,
//     input_length / target_length int64, utt_id bytes);
//   * tf.io.TFRecordWriter + tf.train.Example(...).SerializeToString()
//     (save_speech_data.py:119-120, 178-186).
// Host code only (plain C++17, no HIP): the data path runs on the CPU and hands
// batches to the device through torch.
#include <cerrno>
#include <cstdarg>
#include <cstdio>
#include <cstring>
#include <string>
#include <vector>

#include "../../../include/srf_data.h"

namespace {

thread_local char t_err[512];

void set_err(const char* fmt, ...) {
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(t_err, sizeof(t_err), fmt, ap);
  va_end(ap);
}

constexpr int kEof = 1;
constexpr int kEArg = -1;
constexpr int kECorrupt = -5;
constexpr int kEExample = -6;

// ---------------------------------------------------------------- CRC-32C
// Reflected Castagnoli polynomial 0x82F63B78, slicing-by-8 tables.
struct Crc32cTables {
  uint32_t t[8][256];
  Crc32cTables() {
    for (uint32_t i = 0; i < 256; ++i) {
      uint32_t c = i;
      for (int k = 0; k < 8; ++k) c = (c & 1) ? (c >> 1) ^ 0x82F63B78u : c >> 1;
      t[0][i] = c;
    }
    for (uint32_t i = 0; i < 256; ++i)
      for (int s = 1; s < 8; ++s) t[s][i] = (t[s - 1][i] >> 8) ^ t[0][t[s - 1][i] & 0xff];
  }
};
const Crc32cTables kCrc;

uint32_t crc32c(const uint8_t* p, size_t n) {
  uint32_t c = 0xFFFFFFFFu;
  while (n >= 8) {
    uint32_t lo, hi;
    memcpy(&lo, p, 4);
    memcpy(&hi, p + 4, 4);
    lo ^= c;
    c = kCrc.t[7][lo & 0xff] ^ kCrc.t[6][(lo >> 8) & 0xff] ^ kCrc.t[5][(lo >> 16) & 0xff] ^ kCrc.t[4][lo >> 24] ^
        kCrc.t[3][hi & 0xff] ^ kCrc.t[2][(hi >> 8) & 0xff] ^ kCrc.t[1][(hi >> 16) & 0xff] ^ kCrc.t[0][hi >> 24];
    p += 8;
    n -= 8;
  }
  while (n--) c = (c >> 8) ^ kCrc.t[0][(c ^ *p++) & 0xff];
  return c ^ 0xFFFFFFFFu;
}

uint32_t mask(uint32_t c) { return ((c >> 15) | (c << 17)) + 0xa282ead8u; }

// ---------------------------------------------------------------- protobuf wire
struct Cursor {
  const uint8_t* p;
  const uint8_t* end;
  bool ok = true;
  bool more() const { return ok && p < end; }
  uint64_t varint() {
    uint64_t v = 0;
    for (int s = 0; s < 64; s += 7) {
      if (p >= end) {
        ok = false;
        return 0;
      }
      const uint8_t b = *p++;
      v |= (uint64_t)(b & 0x7f) << s;
      if (!(b & 0x80)) return v;
    }
    ok = false;
    return 0;
  }
  Cursor sub(uint64_t len) {
    Cursor c{p, p};
    if ((uint64_t)(end - p) < len) {
      ok = false;
      return c;
    }
    c.end = p + len;
    p += len;
    return c;
  }
  void skip(int wire) {
    switch (wire) {
      case 0: varint(); break;
      case 1: if (end - p < 8) ok = false; else p += 8; break;
      case 2: sub(varint()); break;
      case 5: if (end - p < 4) ok = false; else p += 4; break;
      default: ok = false;
    }
  }
};

enum Kind { kNone, kBytes, kFloat, kInt64 };

// One Feature message: collects its list (packed or unpacked) into the vectors.
bool parse_feature(Cursor c, Kind& kind, std::vector<float>& fv, std::vector<int64_t>& iv, std::string& bv) {
  kind = kNone;
  while (c.more()) {
    const uint64_t tag = c.varint();
    const int field = (int)(tag >> 3), wire = (int)(tag & 7);
    if (wire != 2 || field < 1 || field > 3) {
      c.skip(wire);
      continue;
    }
    Cursor list = c.sub(c.varint());
    kind = field == 1 ? kBytes : field == 2 ? kFloat : kInt64;
    while (list.more()) {
      const uint64_t lt = list.varint();
      const int lf = (int)(lt >> 3), lw = (int)(lt & 7);
      if (lf != 1) {
        list.skip(lw);
        continue;
      }
      if (kind == kFloat) {
        if (lw == 2) {   // packed
          Cursor pk = list.sub(list.varint());
          if ((pk.end - pk.p) % 4) return false;
          const size_t n = (pk.end - pk.p) / 4, o = fv.size();
          fv.resize(o + n);
          memcpy(fv.data() + o, pk.p, n * 4);
        } else if (lw == 5) {
          if (list.end - list.p < 4) return false;
          float f;
          memcpy(&f, list.p, 4);
          list.p += 4;
          fv.push_back(f);
        } else {
          return false;
        }
      } else if (kind == kInt64) {
        if (lw == 2) {
          Cursor pk = list.sub(list.varint());
          while (pk.more()) iv.push_back((int64_t)pk.varint());
          if (!pk.ok) return false;
        } else if (lw == 0) {
          iv.push_back((int64_t)list.varint());
        } else {
          return false;
        }
      } else {
        if (lw != 2) return false;
        Cursor b = list.sub(list.varint());
        bv.assign(reinterpret_cast<const char*>(b.p), b.end - b.p);
      }
    }
    if (!list.ok) return false;
  }
  return c.ok;
}

struct Handle {
  FILE* f = nullptr;
  bool verify = true;
  std::vector<uint8_t> rec;
  std::vector<float> feats;
  std::vector<int64_t> labels, tmp;
  std::string utt, key, sval;
};

int parse_example(Handle* h, const uint8_t* data, size_t n, srf_speech_example* out) {
  h->feats.clear();
  h->labels.clear();
  h->utt.clear();
  int64_t in_len = -1, tar_len = -1;
  bool have_utt = false;
  Cursor ex{data, data + n};
  while (ex.more()) {
    const uint64_t tag = ex.varint();
    if ((tag >> 3) != 1 || (tag & 7) != 2) {   // Example.features = 1
      ex.skip((int)(tag & 7));
      continue;
    }
    Cursor feats = ex.sub(ex.varint());
    while (feats.more()) {
      const uint64_t ft = feats.varint();
      if ((ft >> 3) != 1 || (ft & 7) != 2) {   // Features.feature = 1 (map entry)
        feats.skip((int)(ft & 7));
        continue;
      }
      Cursor entry = feats.sub(feats.varint());
      h->key.clear();
      Cursor value{nullptr, nullptr};
      bool have_value = false;
      while (entry.more()) {
        const uint64_t et = entry.varint();
        if ((et & 7) != 2) {
          entry.skip((int)(et & 7));
          continue;
        }
        Cursor v = entry.sub(entry.varint());
        if ((et >> 3) == 1) {
          h->key.assign(reinterpret_cast<const char*>(v.p), v.end - v.p);
        } else if ((et >> 3) == 2) {
          value = v;
          have_value = true;
        }
      }
      if (!entry.ok) break;
      if (!have_value) continue;
      Kind kind;
      std::vector<float> fv;
      h->tmp.clear();
      h->sval.clear();
      if (h->key == "input_speech") {
        if (!parse_feature(value, kind, h->feats, h->tmp, h->sval) || (kind != kFloat && kind != kNone)) {
          set_err("input_speech is not a float list");
          return kEExample;
        }
      } else if (h->key == "target_label") {
        if (!parse_feature(value, kind, fv, h->labels, h->sval) || (kind != kInt64 && kind != kNone)) {
          set_err("target_label is not an int64 list");
          return kEExample;
        }
      } else if (h->key == "input_length" || h->key == "target_length") {
        if (!parse_feature(value, kind, fv, h->tmp, h->sval) || kind != kInt64 || h->tmp.size() != 1) {
          set_err("%s must be a single int64 (FixedLenFeature shape ())", h->key.c_str());
          return kEExample;
        }
        (h->key == "input_length" ? in_len : tar_len) = h->tmp[0];
      } else if (h->key == "utt_id") {
        if (!parse_feature(value, kind, fv, h->tmp, h->utt) || kind != kBytes) {
          set_err("utt_id is not a bytes list");
          return kEExample;
        }
        have_utt = true;
      }
    }
    if (!feats.ok) {
      set_err("truncated Features message");
      return kEExample;
    }
  }
  if (!ex.ok) {
    set_err("truncated Example message");
    return kEExample;
  }
  out->input_speech = h->feats.data();
  out->n_input_speech = (int64_t)h->feats.size();
  out->target_label = h->labels.data();
  out->n_target_label = (int64_t)h->labels.size();
  out->input_length = in_len;
  out->target_length = tar_len;
  out->utt_id = have_utt ? h->utt.data() : nullptr;
  out->utt_id_len = have_utt ? (int64_t)h->utt.size() : 0;
  return 0;
}

// ---------------------------------------------------------------- encoding
void put_varint(std::string& s, uint64_t v) {
  while (v >= 0x80) {
    s.push_back((char)(v | 0x80));
    v >>= 7;
  }
  s.push_back((char)v);
}
void put_len(std::string& s, int field, const std::string& body) {
  put_varint(s, ((uint64_t)field << 3) | 2);
  put_varint(s, body.size());
  s += body;
}
std::string feature_float(const float* v, int64_t n) {
  std::string packed(reinterpret_cast<const char*>(v), (size_t)n * 4), list, feat;
  if (n > 0) put_len(list, 1, packed);
  put_len(feat, 2, list);
  return feat;
}
std::string feature_int64(const int64_t* v, int64_t n) {
  std::string packed, list, feat;
  for (int64_t i = 0; i < n; ++i) put_varint(packed, (uint64_t)v[i]);
  if (n > 0) put_len(list, 1, packed);
  put_len(feat, 3, list);
  return feat;
}
std::string feature_bytes(const char* v, int64_t n) {
  std::string list, feat;
  put_len(list, 1, std::string(v, (size_t)n));
  put_len(feat, 1, list);
  return feat;
}
void put_entry(std::string& features, const char* key, const std::string& feature) {
  std::string entry;
  put_len(entry, 1, key);
  put_len(entry, 2, feature);
  put_len(features, 1, entry);
}

}  // namespace

extern "C" {

const char* srf_data_last_error(void) { return t_err; }

uint32_t srf_crc32c(const void* data, size_t n) { return crc32c(static_cast<const uint8_t*>(data), n); }
uint32_t srf_crc32c_masked(const void* data, size_t n) { return mask(srf_crc32c(data, n)); }

void* srf_tfr_open(const char* path, int verify_crc) {
  if (!path) {
    set_err("null path");
    return nullptr;
  }
  FILE* f = fopen(path, "rb");
  if (!f) {
    set_err("cannot open %s: %s", path, strerror(errno));
    return nullptr;
  }
  Handle* h = new Handle;
  h->f = f;
  h->verify = verify_crc != 0;
  return h;
}

void* srf_example_parser_new(void) { return new Handle; }

int srf_tfr_next(void* reader, srf_speech_example* out) {
  Handle* h = static_cast<Handle*>(reader);
  if (!h || !h->f || !out) {
    set_err("bad reader or output");
    return kEArg;
  }
  uint8_t hdr[12];
  const size_t got = fread(hdr, 1, 12, h->f);
  if (got == 0 && feof(h->f)) return kEof;
  if (got != 12) {
    set_err("truncated record header");
    return kECorrupt;
  }
  uint64_t len;
  uint32_t lcrc;
  memcpy(&len, hdr, 8);
  memcpy(&lcrc, hdr + 8, 4);
  if (h->verify && mask(crc32c(hdr, 8)) != lcrc) {
    set_err("length CRC mismatch");
    return kECorrupt;
  }
  if (len > (1ull << 34)) {
    set_err("record length %llu implausible", (unsigned long long)len);
    return kECorrupt;
  }
  h->rec.resize(len);
  uint32_t dcrc;
  if (fread(h->rec.data(), 1, len, h->f) != len || fread(&dcrc, 1, 4, h->f) != 4) {
    set_err("truncated record body");
    return kECorrupt;
  }
  if (h->verify && mask(crc32c(h->rec.data(), len)) != dcrc) {
    set_err("data CRC mismatch");
    return kECorrupt;
  }
  return parse_example(h, h->rec.data(), len, out);
}

const uint8_t* srf_tfr_record(void* reader, size_t* n) {
  Handle* h = static_cast<Handle*>(reader);
  if (!h) return nullptr;
  if (n) *n = h->rec.size();
  return h->rec.data();
}

int srf_example_parse(void* handle, const uint8_t* data, size_t n, srf_speech_example* out) {
  Handle* h = static_cast<Handle*>(handle);
  if (!h || (!data && n) || !out) {
    set_err("bad arguments");
    return kEArg;
  }
  return parse_example(h, data, n, out);
}

int srf_tfr_close(void* reader) {
  Handle* h = static_cast<Handle*>(reader);
  if (!h) return kEArg;
  if (h->f) fclose(h->f);
  delete h;
  return 0;
}

void* srf_tfr_writer_open(const char* path) {
  FILE* f = path ? fopen(path, "wb") : nullptr;
  if (!f) {
    set_err("cannot create %s: %s", path ? path : "(null)", strerror(errno));
    return nullptr;
  }
  Handle* h = new Handle;
  h->f = f;
  return h;
}

int srf_tfr_write_record(void* writer, const uint8_t* data, size_t n) {
  Handle* h = static_cast<Handle*>(writer);
  if (!h || !h->f || (!data && n)) {
    set_err("bad writer");
    return kEArg;
  }
  uint8_t hdr[12];
  const uint64_t len = n;
  memcpy(hdr, &len, 8);
  const uint32_t lcrc = mask(crc32c(hdr, 8)), dcrc = mask(crc32c(data, n));
  memcpy(hdr + 8, &lcrc, 4);
  if (fwrite(hdr, 1, 12, h->f) != 12 || fwrite(data, 1, n, h->f) != n || fwrite(&dcrc, 1, 4, h->f) != 4) {
    set_err("write failed: %s", strerror(errno));
    return kEArg;
  }
  return 0;
}

int srf_tfr_write_example(void* writer, const float* input_speech, int64_t n_input_speech,
                          const int64_t* target_label, int64_t n_target_label, int64_t input_length,
                          int64_t target_length, const char* utt_id, int64_t utt_id_len) {
  if (n_input_speech < 0 || n_target_label < 0 || (n_input_speech && !input_speech) ||
      (n_target_label && !target_label)) {
    set_err("bad example arguments");
    return kEArg;
  }
  // map entries in key order = protobuf's deterministic map serialisation
  std::string features, example;
  put_entry(features, "input_length", feature_int64(&input_length, 1));
  put_entry(features, "input_speech", feature_float(input_speech, n_input_speech));
  put_entry(features, "target_label", feature_int64(target_label, n_target_label));
  put_entry(features, "target_length", feature_int64(&target_length, 1));
  if (utt_id) put_entry(features, "utt_id", feature_bytes(utt_id, utt_id_len));
  put_len(example, 1, features);
  return srf_tfr_write_record(writer, reinterpret_cast<const uint8_t*>(example.data()), example.size());
}

int srf_tfr_writer_close(void* writer) { return srf_tfr_close(writer); }

}  // extern "C"
