// wire.cpp -- DRW1 capture reader (include/dagrider_wire.h): parse, check every
// size and offset, then hand the arrays to dr_append_rounds_lists.  Host code
// only; the same checks as dag_rider_amd/wire.py _parse.
#include <cstring>
#include <vector>

#include "dagrider_wire.h"

namespace {

struct View {
  const uint8_t *p = nullptr;
  size_t len = 0, pos = 0;
  bool take(size_t n, const uint8_t **out) {
    if (n > len - pos) return false;
    *out = p + pos;
    pos += n;
    return true;
  }
  bool u64(uint64_t *v) {
    const uint8_t *q;
    if (!take(8, &q)) return false;
    std::memcpy(v, q, 8);
    return true;
  }
};

struct Capture {
  uint32_t nrounds = 0, nslots = 0;
  const uint32_t *so = nullptr, *sto = nullptr, *wo = nullptr;
  const int32_t *sid = nullptr, *sti = nullptr, *wi = nullptr;
  uint64_t nsti = 0, nwi = 0;
  const uint8_t *boff = nullptr, *blocks = nullptr;
};

// a u32 offset array of n+1 entries: 0-based, non-decreasing, ending at total
bool offsets_ok(const uint32_t *o, uint64_t n, uint64_t total) {
  uint32_t prev = 0;
  for (uint64_t i = 0; i <= n; i++) {
    uint32_t x;
    std::memcpy(&x, o + i, 4);  // the buffer need not be 4-aligned
    if ((i == 0 && x != 0) || x < prev) return false;
    prev = x;
  }
  return prev == total;
}

int parse(const void *buf, size_t len, Capture *c) {
  if (!buf) return DR_E_INVAL;
  View v;
  v.p = static_cast<const uint8_t *>(buf);
  v.len = len;
  const uint8_t *h;
  if (!v.take(12, &h) || std::memcmp(h, "DRW1", 4) != 0) return DR_E_INVAL;
  std::memcpy(&c->nrounds, h + 4, 4);
  std::memcpy(&c->nslots, h + 8, 4);
  const uint8_t *arr[6];
  uint64_t cnt[6];
  for (int i = 0; i < 6; i++) {
    if (!v.u64(&cnt[i]) || cnt[i] > (v.len - v.pos) / 4 || !v.take(cnt[i] * 4, &arr[i])) return DR_E_INVAL;
  }
  if (cnt[0] != (uint64_t)c->nrounds + 1 || cnt[1] != 2ull * c->nslots || cnt[2] != (uint64_t)c->nslots + 1 ||
      cnt[4] != (uint64_t)c->nslots + 1 || (cnt[3] & 1) || (cnt[5] & 1))
    return DR_E_INVAL;
  c->so = reinterpret_cast<const uint32_t *>(arr[0]);
  c->sid = reinterpret_cast<const int32_t *>(arr[1]);
  c->sto = reinterpret_cast<const uint32_t *>(arr[2]);
  c->sti = reinterpret_cast<const int32_t *>(arr[3]);
  c->wo = reinterpret_cast<const uint32_t *>(arr[4]);
  c->wi = reinterpret_cast<const int32_t *>(arr[5]);
  c->nsti = cnt[3] / 2;
  c->nwi = cnt[5] / 2;
  if (!offsets_ok(c->so, c->nrounds, c->nslots) || !offsets_ok(c->sto, c->nslots, c->nsti) ||
      !offsets_ok(c->wo, c->nslots, c->nwi))
    return DR_E_INVAL;
  if (!v.take(8ull * ((uint64_t)c->nslots + 1), &c->boff)) return DR_E_INVAL;
  uint64_t prev = 0;
  for (uint64_t i = 0; i <= c->nslots; i++) {
    uint64_t x;
    std::memcpy(&x, c->boff + 8 * i, 8);
    if ((i == 0 && x != 0) || x < prev) return DR_E_INVAL;
    prev = x;
  }
  if (prev != v.len - v.pos) return DR_E_INVAL;  // block bytes exactly fill the rest
  c->blocks = v.p + v.pos;
  return DR_OK;
}

}  // namespace

extern "C" int dr_wire_check(const void *buf, size_t len, int32_t *nrounds, int32_t *nslots) {
  Capture c;
  if (int rc = parse(buf, len, &c)) return rc;
  if (nrounds) *nrounds = (int32_t)c.nrounds;
  if (nslots) *nslots = (int32_t)c.nslots;
  return DR_OK;
}

extern "C" int dr_wire_append(dr_ctx *ctx, const void *buf, size_t len) {
  if (!ctx) return DR_E_INVAL;
  Capture c;
  if (int rc = parse(buf, len, &c)) return rc;
  if (c.nrounds == 0) return DR_OK;
  // the arrays may sit at any alignment inside buf: copy them to aligned storage
  auto copy = [](const void *src, size_t n, std::vector<int32_t> &dst) {
    dst.resize(n ? n : 1, 0);
    if (n) std::memcpy(dst.data(), src, n * 4);
    return dst.data();
  };
  std::vector<int32_t> so, sid, sto, sti, wo, wi;
  copy(c.so, (size_t)c.nrounds + 1, so);
  copy(c.sid, 2 * (size_t)c.nslots, sid);
  copy(c.sto, (size_t)c.nslots + 1, sto);
  copy(c.sti, 2 * (size_t)c.nsti, sti);
  copy(c.wo, (size_t)c.nslots + 1, wo);
  copy(c.wi, 2 * (size_t)c.nwi, wi);
  return dr_append_rounds_lists(ctx, dr_num_rounds(ctx), (int)c.nrounds, reinterpret_cast<const uint32_t *>(so.data()),
                                sid.data(), reinterpret_cast<const uint32_t *>(sto.data()), sti.data(),
                                reinterpret_cast<const uint32_t *>(wo.data()), wi.data());
}

extern "C" int dr_wire_block(const void *buf, size_t len, int64_t slot, const uint8_t **data, size_t *n) {
  Capture c;
  if (int rc = parse(buf, len, &c)) return rc;
  if (slot < 0 || slot >= (int64_t)c.nslots || !data || !n) return DR_E_INVAL;
  uint64_t a, b;
  std::memcpy(&a, c.boff + 8 * slot, 8);
  std::memcpy(&b, c.boff + 8 * (slot + 1), 8);
  *data = c.blocks + a;
  *n = (size_t)(b - a);
  return DR_OK;
}
