// mraft_persist.cpp — host-only codec of one replica's persistent state
// (include/mraft.h mraft_encode_persistent / mraft_decode_persistent): the
// bytes a Persister holds for SaveState (src/raft/raft.go:209-216) /
// readPersist (:217-235). Not gob: a fixed little-endian layout
//   "MRPS" | u32 version | i64 currentTerm | i64 votedFor | i64 dummyIndex |
//   u32 count | count x i64 term
// (Go's int is 64-bit, so the wire keeps 64-bit fields). Commands are not
// engine state: the host stores them next to these bytes, index-aligned.
#include <cstring>

#include "../../include/mraft.h"

namespace {

constexpr uint32_t kVersion = 1;
constexpr int64_t kHeader = 4 + 4 + 8 + 8 + 8 + 4;

void put_u32(uint8_t *p, uint32_t v) {
  for (int i = 0; i < 4; ++i) p[i] = (uint8_t)(v >> (8 * i));
}
void put_i64(uint8_t *p, int64_t v) {
  for (int i = 0; i < 8; ++i) p[i] = (uint8_t)((uint64_t)v >> (8 * i));
}
uint32_t get_u32(const uint8_t *p) {
  uint32_t v = 0;
  for (int i = 0; i < 4; ++i) v |= (uint32_t)p[i] << (8 * i);
  return v;
}
int64_t get_i64(const uint8_t *p) {
  uint64_t v = 0;
  for (int i = 0; i < 8; ++i) v |= (uint64_t)p[i] << (8 * i);
  return (int64_t)v;
}
bool fits_i32(int64_t v) { return v >= INT32_MIN && v <= INT32_MAX; }

}  // namespace

extern "C" {

int64_t mraft_encode_persistent(const mraft_persistent *in, const int32_t *terms, uint8_t *out,
                                int64_t cap) {
  if (!in) return MRAFT_E_INVAL;
  const int64_t count = (int64_t)in->last_index - in->dummy_index + 1;
  if (count < 1 || count > UINT32_MAX || in->terms_offset < 0 || !terms) return MRAFT_E_INVAL;
  const int64_t size = kHeader + 8 * count;
  if (!out || cap < size) return size;
  std::memcpy(out, "MRPS", 4);
  put_u32(out + 4, kVersion);
  put_i64(out + 8, in->current_term);
  put_i64(out + 16, in->voted_for);
  put_i64(out + 24, in->dummy_index);
  put_u32(out + 32, (uint32_t)count);
  const int32_t *t = terms + in->terms_offset;
  for (int64_t k = 0; k < count; ++k) put_i64(out + kHeader + 8 * k, t[k]);
  return size;
}

int mraft_decode_persistent(const uint8_t *buf, int64_t len, mraft_persistent *out, int32_t *terms,
                            int64_t terms_cap) {
  if (!buf || !out || len < kHeader || std::memcmp(buf, "MRPS", 4) != 0 ||
      get_u32(buf + 4) != kVersion)
    return MRAFT_E_INVAL;
  const int64_t term = get_i64(buf + 8), voted = get_i64(buf + 16), dummy = get_i64(buf + 24);
  const int64_t count = get_u32(buf + 32);
  if (count < 1 || len != kHeader + 8 * count || !fits_i32(term) || !fits_i32(voted) ||
      !fits_i32(dummy) || !fits_i32(dummy + count - 1) || terms_cap < count || !terms)
    return MRAFT_E_INVAL;
  for (int64_t k = 0; k < count; ++k) {
    const int64_t t = get_i64(buf + kHeader + 8 * k);
    if (!fits_i32(t)) return MRAFT_E_INVAL;
    terms[k] = (int32_t)t;
  }
  out->current_term = (int32_t)term;
  out->voted_for = (int32_t)voted;
  out->dummy_index = (int32_t)dummy;
  out->last_index = (int32_t)(dummy + count - 1);
  out->_pad = 0;
  out->terms_offset = 0;
  return MRAFT_OK;
}

}  // extern "C"
