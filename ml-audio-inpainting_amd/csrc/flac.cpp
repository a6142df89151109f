// flac.cpp — native FLAC decoder (host code), SURVEY §8 f2.
//
// Replaces the soundfile/libsndfile decode behind utils.load_audio ->
// librosa.load (utils.py:36) for the LibriSpeech FLAC clips the reference
// trains on (models/CNNBLSTM/dataset.py:95, models/GAN/dataset.py:80-84).
// Follows the FLAC format specification (RFC 9639): STREAMINFO, frame headers
// (CRC-8), CONSTANT / VERBATIM / FIXED (orders 0-4) / LPC subframes with
// wasted bits, Rice / Rice2 partitioned residuals incl. escape partitions,
// independent and left/side, side/right, mid/side stereo decorrelation, frame
// CRC-16.  Output: interleaved signed integer samples, exactly as encoded;
// the STREAMINFO MD5 of those samples is the bit-exactness check
// (tests/test_cpu_flac.py).  The reference decodes each file 2*G times per
// item (utils.py:36,168); the build decodes it once.
#include <stdint.h>
#include <stdio.h>
#include <string.h>

#include <vector>

#include "../../include/ainp.h"

namespace ainp {
int record_msg(const char* msg);
}

namespace {

struct Bits {
  const uint8_t* p;
  size_t n;       // bytes
  size_t pos = 0; // bit position
  bool bad = false;

  uint64_t get(int k) {  // k <= 57
    if (k == 0) return 0;
    if (pos + (size_t)k > n * 8) {
      bad = true;
      pos = n * 8;
      return 0;
    }
    uint64_t v = 0;
    for (int i = 0; i < k;) {
      const size_t byte = pos >> 3;
      const int off = (int)(pos & 7);
      const int take = (8 - off) < (k - i) ? (8 - off) : (k - i);
      const uint64_t chunk = (p[byte] >> (8 - off - take)) & ((1u << take) - 1);
      v = (v << take) | chunk;
      pos += take;
      i += take;
    }
    return v;
  }
  int64_t sget(int k) {  // two's complement, k <= 57
    if (k == 0) return 0;
    const uint64_t v = get(k);
    return (int64_t)(v << (64 - k)) >> (64 - k);
  }
  uint32_t unary() {  // number of 0 bits before the next 1
    uint32_t q = 0;
    while (true) {
      if (pos >= n * 8) {
        bad = true;
        return q;
      }
      const size_t byte = pos >> 3;
      const int off = (int)(pos & 7);
      const uint8_t rest = (uint8_t)(p[byte] << off);
      if (rest) {
        const int lz = __builtin_clz((uint32_t)rest) - 24;
        q += lz;
        pos += lz + 1;
        return q;
      }
      q += 8 - off;
      pos += 8 - off;
    }
  }
  void align() { pos = (pos + 7) & ~(size_t)7; }
};

uint8_t crc8(const uint8_t* d, size_t n) {
  uint8_t c = 0;
  for (size_t i = 0; i < n; ++i) {
    c ^= d[i];
    for (int b = 0; b < 8; ++b) c = (uint8_t)((c & 0x80) ? (c << 1) ^ 0x07 : (c << 1));
  }
  return c;
}

uint16_t crc16(const uint8_t* d, size_t n) {
  uint16_t c = 0;
  for (size_t i = 0; i < n; ++i) {
    c ^= (uint16_t)(d[i] << 8);
    for (int b = 0; b < 8; ++b) c = (uint16_t)((c & 0x8000) ? (c << 1) ^ 0x8005 : (c << 1));
  }
  return c;
}

struct StreamInfo {
  int min_block = 0, max_block = 0, sample_rate = 0, channels = 0, bps = 0;
  int64_t total = 0;
  uint8_t md5[16] = {0};
  size_t frames_at = 0;  // byte offset of the first frame
};

int fail(const char* m) { return ainp::record_msg(m); }

// Predictor / decorrelation arithmetic wraps modulo 2^64 like the hardware
// does: a valid stream never leaves the sample range (so the results are the
// same), and a corrupted one cannot hit signed-overflow UB (found by the UBSan
// harness, tests/sanitize/flac_fuzz.cpp); its CRC-16 check rejects it later.
inline int64_t wadd(int64_t a, int64_t b) { return (int64_t)((uint64_t)a + (uint64_t)b); }
inline int64_t wsub(int64_t a, int64_t b) { return (int64_t)((uint64_t)a - (uint64_t)b); }
inline int64_t wmul(int64_t a, int64_t b) { return (int64_t)((uint64_t)a * (uint64_t)b); }

int parse_header(const uint8_t* d, size_t n, StreamInfo& si) {
  size_t at = 0;
  if (n >= 10 && d[0] == 'I' && d[1] == 'D' && d[2] == '3') {  // ID3v2 tag in front
    const size_t sz = ((size_t)(d[6] & 0x7f) << 21) | ((size_t)(d[7] & 0x7f) << 14) |
                      ((size_t)(d[8] & 0x7f) << 7) | (size_t)(d[9] & 0x7f);
    at = 10 + sz;
  }
  if (n < at + 4 || memcmp(d + at, "fLaC", 4) != 0) return fail("flac: missing fLaC marker");
  at += 4;
  bool have_info = false;
  while (true) {
    if (at + 4 > n) return fail("flac: truncated metadata");
    const bool last = d[at] & 0x80;
    const int type = d[at] & 0x7f;
    const size_t len = ((size_t)d[at + 1] << 16) | ((size_t)d[at + 2] << 8) | d[at + 3];
    at += 4;
    if (at + len > n) return fail("flac: truncated metadata block");
    if (type == 0) {
      if (len < 34) return fail("flac: short STREAMINFO");
      Bits b{d + at, len};
      si.min_block = (int)b.get(16);
      si.max_block = (int)b.get(16);
      b.get(24);
      b.get(24);
      si.sample_rate = (int)b.get(20);
      si.channels = (int)b.get(3) + 1;
      si.bps = (int)b.get(5) + 1;
      si.total = (int64_t)b.get(36);
      memcpy(si.md5, d + at + 18, 16);
      have_info = true;
    }
    at += len;
    if (last) break;
  }
  if (!have_info) return fail("flac: no STREAMINFO");
  if (si.bps < 4 || si.bps > 32) return fail("flac: unsupported bits per sample");
  si.frames_at = at;
  return AINP_OK;
}

// Rice-coded residual of one subframe into res[order..blocksize)
bool residual(Bits& b, int blocksize, int order, int64_t* res) {
  const int method = (int)b.get(2);
  if (method > 1) return false;
  const int pbits = method == 0 ? 4 : 5, esc = method == 0 ? 15 : 31;
  const int porder = (int)b.get(4);
  const int parts = 1 << porder;
  if ((blocksize >> porder) < order || (blocksize & (parts - 1))) return false;
  int i = order;
  for (int pt = 0; pt < parts; ++pt) {
    const int cnt = (blocksize >> porder) - (pt == 0 ? order : 0);
    const int k = (int)b.get(pbits);
    if (k == esc) {
      const int nb = (int)b.get(5);
      for (int j = 0; j < cnt; ++j) res[i++] = b.sget(nb);
    } else {
      for (int j = 0; j < cnt; ++j) {
        const uint64_t q = b.unary();
        const uint64_t u = (q << k) | b.get(k);
        res[i++] = (int64_t)(u >> 1) ^ -(int64_t)(u & 1);
      }
    }
    if (b.bad) return false;
  }
  return true;
}

bool subframe(Bits& b, int blocksize, int bps, int64_t* out) {
  if (b.get(1) != 0) return false;  // zero pad bit
  const int type = (int)b.get(6);
  int wasted = 0;
  if (b.get(1)) wasted = (int)b.unary() + 1;
  bps -= wasted;
  if (bps <= 0) return false;
  if (type == 0) {  // CONSTANT
    const int64_t v = b.sget(bps);
    for (int i = 0; i < blocksize; ++i) out[i] = v;
  } else if (type == 1) {  // VERBATIM
    for (int i = 0; i < blocksize; ++i) out[i] = b.sget(bps);
  } else if (type >= 8 && type <= 12) {  // FIXED, order 0..4
    const int order = type - 8;
    if (order > blocksize) return false;
    for (int i = 0; i < order; ++i) out[i] = b.sget(bps);
    if (!residual(b, blocksize, order, out)) return false;
    for (int i = order; i < blocksize; ++i) {
      int64_t pred = 0;
      switch (order) {
        case 1: pred = out[i - 1]; break;
        case 2: pred = wsub(wmul(2, out[i - 1]), out[i - 2]); break;
        case 3:
          pred = wadd(wsub(wmul(3, out[i - 1]), wmul(3, out[i - 2])), out[i - 3]);
          break;
        case 4:
          pred = wsub(wadd(wsub(wmul(4, out[i - 1]), wmul(6, out[i - 2])), wmul(4, out[i - 3])),
                      out[i - 4]);
          break;
        default: break;
      }
      out[i] = wadd(out[i], pred);
    }
  } else if (type >= 32) {  // LPC, order 1..32
    const int order = type - 31;
    if (order > blocksize) return false;
    for (int i = 0; i < order; ++i) out[i] = b.sget(bps);
    const int prec = (int)b.get(4) + 1;
    if (prec == 16) return false;  // 0b1111 is invalid
    const int shift = (int)b.sget(5);
    if (shift < 0) return false;
    int64_t coef[32];
    for (int j = 0; j < order; ++j) coef[j] = b.sget(prec);
    if (!residual(b, blocksize, order, out)) return false;
    for (int i = order; i < blocksize; ++i) {
      int64_t sum = 0;
      for (int j = 0; j < order; ++j) sum = wadd(sum, wmul(coef[j], out[i - 1 - j]));
      out[i] = wadd(out[i], sum >> shift);
    }
  } else {
    return false;  // reserved
  }
  if (wasted)
    for (int i = 0; i < blocksize; ++i) out[i] = (int64_t)((uint64_t)out[i] << wasted);
  return !b.bad;
}

}  // namespace

extern "C" int ainp_flac_info(const uint8_t* data, size_t n, int* sample_rate, int* channels,
                              int* bits_per_sample, int64_t* total_samples, uint8_t* md5) {
  if (!data) return fail("ainp_flac_info: bad argument");
  StreamInfo si;
  const int rc = parse_header(data, n, si);
  if (rc) return rc;
  if (sample_rate) *sample_rate = si.sample_rate;
  if (channels) *channels = si.channels;
  if (bits_per_sample) *bits_per_sample = si.bps;
  if (total_samples) *total_samples = si.total;
  if (md5) memcpy(md5, si.md5, 16);
  return AINP_OK;
}

extern "C" int ainp_flac_decode(const uint8_t* data, size_t n, int32_t* out, int64_t max_frames,
                                int64_t* n_frames) {
  if (!data || !out || max_frames < 0 || !n_frames) return fail("ainp_flac_decode: bad argument");
  StreamInfo si;
  int rc = parse_header(data, n, si);
  if (rc) return rc;
  const int nch = si.channels;
  std::vector<int64_t> ch[8];
  int64_t done = 0;
  size_t at = si.frames_at;
  while (at + 2 <= n && (si.total == 0 || done < si.total)) {
    // ---- frame header
    if (data[at] != 0xFF || (data[at + 1] & 0xFE) != 0xF8) return fail("flac: lost frame sync");
    Bits b{data + at, n - at};
    b.get(15);
    b.get(1);  // blocking strategy (the sample number below is not needed)
    const int bs_code = (int)b.get(4), sr_code = (int)b.get(4);
    const int ch_code = (int)b.get(4), ss_code = (int)b.get(3);
    b.get(1);
    {  // UTF-8-like coded frame / sample number
      const uint64_t first = b.get(8);
      int extra = 0;
      if (first & 0x80) {
        uint64_t m = 0x40;
        while (first & m) {
          ++extra;
          m >>= 1;
        }
        if (extra == 0 || extra > 6) return fail("flac: bad coded number");
      }
      for (int i = 0; i < extra; ++i)
        if ((b.get(8) & 0xC0) != 0x80) return fail("flac: bad coded number");
    }
    int blocksize;
    if (bs_code == 0) return fail("flac: reserved block size");
    else if (bs_code == 1) blocksize = 192;
    else if (bs_code <= 5) blocksize = 576 << (bs_code - 2);
    else if (bs_code == 6) blocksize = (int)b.get(8) + 1;
    else if (bs_code == 7) blocksize = (int)b.get(16) + 1;
    else blocksize = 256 << (bs_code - 8);
    if (sr_code == 12) b.get(8);
    else if (sr_code == 13 || sr_code == 14) b.get(16);
    else if (sr_code == 15) return fail("flac: invalid sample rate code");
    int bps = si.bps;
    static const int ss_tab[8] = {0, 8, 12, 0, 16, 20, 24, 32};
    if (ss_code == 3) return fail("flac: reserved sample size");
    if (ss_code) bps = ss_tab[ss_code];
    const size_t hdr_bytes = b.pos / 8;
    const uint8_t crc = (uint8_t)b.get(8);
    if (b.bad || crc != crc8(data + at, hdr_bytes)) return fail("flac: frame header CRC-8 mismatch");
    int fch;
    if (ch_code < 8) fch = ch_code + 1;
    else if (ch_code <= 10) fch = 2;
    else return fail("flac: reserved channel assignment");
    if (fch != nch) return fail("flac: channel count changes");
    // ---- subframes
    for (int c = 0; c < fch; ++c) {
      ch[c].assign(blocksize, 0);
      int sbps = bps;
      if ((ch_code == 8 && c == 1) || (ch_code == 9 && c == 0) || (ch_code == 10 && c == 1))
        ++sbps;  // side channel
      if (!subframe(b, blocksize, sbps, ch[c].data())) return fail("flac: bad subframe");
    }
    if (ch_code == 8) {
      for (int i = 0; i < blocksize; ++i) ch[1][i] = wsub(ch[0][i], ch[1][i]);
    } else if (ch_code == 9) {
      for (int i = 0; i < blocksize; ++i) ch[0][i] = wadd(ch[0][i], ch[1][i]);
    } else if (ch_code == 10) {
      for (int i = 0; i < blocksize; ++i) {
        const int64_t side = ch[1][i];
        const int64_t mid = wmul(ch[0][i], 2) | (side & 1);
        ch[0][i] = wadd(mid, side) >> 1;
        ch[1][i] = wsub(mid, side) >> 1;
      }
    }
    b.align();
    const size_t body = b.pos / 8;
    const uint16_t fcrc = (uint16_t)b.get(16);
    if (b.bad || fcrc != crc16(data + at, body)) return fail("flac: frame CRC-16 mismatch");
    int take = blocksize;
    if (si.total && done + take > si.total) take = (int)(si.total - done);
    if (done + take > max_frames) return fail("flac: output buffer too small");
    for (int i = 0; i < take; ++i)
      for (int c = 0; c < nch; ++c) out[(done + i) * nch + c] = (int32_t)ch[c][i];
    done += take;
    at += b.pos / 8;
  }
  if (si.total && done != si.total) return fail("flac: stream ended early");
  *n_frames = done;
  return AINP_OK;
}

// ============================================================== encoder
// Writer behind utils.save_audio (utils.py:54-89, soundfile.write(...,'FLAC')
// PCM_16) for add_gaps.py / pre_process_dataset.py.  RFC 9639
// subset: STREAMINFO with the MD5 of the samples, fixed 4096-sample blocks
// (a shorter last one), independent channels; per subframe the cheapest of
// CONSTANT, FIXED orders 0-4 with partitioned Rice residuals (partition order
// and parameters chosen by exact bit count) and VERBATIM.  Lossless: the
// decoder above returns the input samples bit for bit (tests/test_cpu_flac.py).
namespace {

struct BitOut {
  std::vector<uint8_t> buf;
  uint64_t acc = 0;
  int nacc = 0;
  void put(uint64_t v, int k) {  // k <= 32
    if (k == 0) return;
    acc = (acc << k) | (v & ((k == 64) ? ~0ull : ((1ull << k) - 1)));
    nacc += k;
    while (nacc >= 8) {
      buf.push_back((uint8_t)(acc >> (nacc - 8)));
      nacc -= 8;
    }
  }
  void sput(int64_t v, int k) { put((uint64_t)v & ((1ull << k) - 1), k); }
  void unary(uint32_t q) {  // q zeros then a one
    while (q >= 32) {
      put(0, 32);
      q -= 32;
    }
    put(1, q + 1);
  }
  void align() {
    if (nacc) put(0, 8 - nacc);
  }
};

// MD5 (RFC 1321) of the samples as FLAC defines it
struct Md5 {
  uint32_t h[4] = {0x67452301u, 0xefcdab89u, 0x98badcfeu, 0x10325476u};
  uint8_t blk[64];
  size_t nb = 0;
  uint64_t len = 0;
  static uint32_t rol(uint32_t x, int c) { return (x << c) | (x >> (32 - c)); }
  void block(const uint8_t* p) {
    static const uint32_t K[64] = {
        0xd76aa478, 0xe8c7b756, 0x242070db, 0xc1bdceee, 0xf57c0faf, 0x4787c62a, 0xa8304613,
        0xfd469501, 0x698098d8, 0x8b44f7af, 0xffff5bb1, 0x895cd7be, 0x6b901122, 0xfd987193,
        0xa679438e, 0x49b40821, 0xf61e2562, 0xc040b340, 0x265e5a51, 0xe9b6c7aa, 0xd62f105d,
        0x02441453, 0xd8a1e681, 0xe7d3fbc8, 0x21e1cde6, 0xc33707d6, 0xf4d50d87, 0x455a14ed,
        0xa9e3e905, 0xfcefa3f8, 0x676f02d9, 0x8d2a4c8a, 0xfffa3942, 0x8771f681, 0x6d9d6122,
        0xfde5380c, 0xa4beea44, 0x4bdecfa9, 0xf6bb4b60, 0xbebfbc70, 0x289b7ec6, 0xeaa127fa,
        0xd4ef3085, 0x04881d05, 0xd9d4d039, 0xe6db99e5, 0x1fa27cf8, 0xc4ac5665, 0xf4292244,
        0x432aff97, 0xab9423a7, 0xfc93a039, 0x655b59c3, 0x8f0ccc92, 0xffeff47d, 0x85845dd1,
        0x6fa87e4f, 0xfe2ce6e0, 0xa3014314, 0x4e0811a1, 0xf7537e82, 0xbd3af235, 0x2ad7d2bb,
        0xeb86d391};
    static const int R[64] = {7, 12, 17, 22, 7, 12, 17, 22, 7, 12, 17, 22, 7, 12, 17, 22,
                              5, 9,  14, 20, 5, 9,  14, 20, 5, 9,  14, 20, 5, 9,  14, 20,
                              4, 11, 16, 23, 4, 11, 16, 23, 4, 11, 16, 23, 4, 11, 16, 23,
                              6, 10, 15, 21, 6, 10, 15, 21, 6, 10, 15, 21, 6, 10, 15, 21};
    uint32_t w[16];
    for (int i = 0; i < 16; ++i)
      w[i] = p[4 * i] | (p[4 * i + 1] << 8) | (p[4 * i + 2] << 16) | ((uint32_t)p[4 * i + 3] << 24);
    uint32_t a = h[0], b = h[1], c = h[2], d = h[3];
    for (int i = 0; i < 64; ++i) {
      uint32_t f;
      int g;
      if (i < 16) { f = (b & c) | (~b & d); g = i; }
      else if (i < 32) { f = (d & b) | (~d & c); g = (5 * i + 1) & 15; }
      else if (i < 48) { f = b ^ c ^ d; g = (3 * i + 5) & 15; }
      else { f = c ^ (b | ~d); g = (7 * i) & 15; }
      const uint32_t t = d;
      d = c;
      c = b;
      b = b + rol(a + f + K[i] + w[g], R[i]);
      a = t;
    }
    h[0] += a; h[1] += b; h[2] += c; h[3] += d;
  }
  void update(const uint8_t* p, size_t n) {
    len += n;
    while (n) {
      const size_t take = (64 - nb) < n ? (64 - nb) : n;
      memcpy(blk + nb, p, take);
      nb += take;
      p += take;
      n -= take;
      if (nb == 64) {
        block(blk);
        nb = 0;
      }
    }
  }
  void final(uint8_t out[16]) {
    const uint64_t bits = len * 8;
    const uint8_t pad = 0x80;
    update(&pad, 1);
    const uint8_t z = 0;
    while (nb != 56) update(&z, 1);
    uint8_t lb[8];
    for (int i = 0; i < 8; ++i) lb[i] = (uint8_t)(bits >> (8 * i));
    update(lb, 8);
    for (int i = 0; i < 4; ++i)
      for (int j = 0; j < 4; ++j) out[4 * i + j] = (uint8_t)(h[i] >> (8 * j));
  }
};

inline uint32_t zigzag(int64_t r) { return (uint32_t)(((uint64_t)r << 1) ^ (uint64_t)(r >> 63)); }

// Exact bits of the Rice-coded residual r[0..n) with the best partition order
// <= max_po (partition 0 shortened by `order` warm-up samples) and per-
// partition parameter <= 14; fills the chosen parameters.
uint64_t rice_plan(const std::vector<uint32_t>& u, int blocksize, int order, int& best_po,
                   std::vector<int>& best_k) {
  uint64_t best = ~0ull;
  int max_po = 0;
  while (max_po < 8 && (blocksize % (2 << max_po)) == 0 && (blocksize >> (max_po + 1)) > order)
    ++max_po;
  for (int po = 0; po <= max_po; ++po) {
    const int np = 1 << po, ps = blocksize >> po;
    uint64_t total = 4 + 4 * (uint64_t)np;   // partition order + parameters
    std::vector<int> ks(np);
    size_t at = 0;
    for (int pi = 0; pi < np; ++pi) {
      const int cnt = pi == 0 ? ps - order : ps;
      uint64_t sum = 0;
      for (int i = 0; i < cnt; ++i) sum += u[at + i];
      uint64_t bestp = ~0ull;
      int bk = 0;
      for (int k = 0; k <= 14; ++k) {
        uint64_t bits = (uint64_t)cnt * (k + 1);
        for (int i = 0; i < cnt; ++i) bits += u[at + i] >> k;
        if (bits < bestp) {
          bestp = bits;
          bk = k;
        }
        if ((sum >> k) == 0) break;
      }
      ks[pi] = bk;
      total += bestp;
      at += cnt;
    }
    if (total < best) {
      best = total;
      best_po = po;
      best_k = ks;
    }
  }
  return best;
}

void write_subframe(BitOut& bo, const int32_t* x, int n, int bps) {
  bool constant = true;
  for (int i = 1; i < n && constant; ++i) constant = x[i] == x[0];
  if (constant) {
    bo.put(0, 1);
    bo.put(0, 6);   // SUBFRAME_CONSTANT
    bo.put(0, 1);   // no wasted bits
    bo.sput(x[0], bps);
    return;
  }
  // FIXED predictors of order 0..4 (when the block is long enough)
  int best_order = -1, best_po = 0;
  uint64_t best_bits = (uint64_t)n * bps;   // VERBATIM
  std::vector<int> best_k;
  std::vector<uint32_t> best_u;
  for (int order = 0; order <= 4 && order < n; ++order) {
    std::vector<uint32_t> u(n - order);
    bool ok = true;
    for (int i = order; i < n; ++i) {
      int64_t r;
      switch (order) {
        case 0: r = x[i]; break;
        case 1: r = (int64_t)x[i] - x[i - 1]; break;
        case 2: r = (int64_t)x[i] - 2 * (int64_t)x[i - 1] + x[i - 2]; break;
        case 3: r = (int64_t)x[i] - 3 * (int64_t)x[i - 1] + 3 * (int64_t)x[i - 2] - x[i - 3]; break;
        default:
          r = (int64_t)x[i] - 4 * (int64_t)x[i - 1] + 6 * (int64_t)x[i - 2] -
              4 * (int64_t)x[i - 3] + x[i - 4];
      }
      if (r > INT32_MAX / 2 || r < -(INT32_MAX / 2)) ok = false;
      u[i - order] = zigzag(r);
    }
    if (!ok) continue;
    int po;
    std::vector<int> ks;
    const uint64_t bits = (uint64_t)order * bps + 2 + rice_plan(u, n, order, po, ks);
    if (bits < best_bits) {
      best_bits = bits;
      best_order = order;
      best_po = po;
      best_k = ks;
      best_u.swap(u);
    }
  }
  bo.put(0, 1);
  if (best_order < 0) {
    bo.put(1, 6);   // SUBFRAME_VERBATIM
    bo.put(0, 1);
    for (int i = 0; i < n; ++i) bo.sput(x[i], bps);
    return;
  }
  bo.put(8 | best_order, 6);   // SUBFRAME_FIXED, order
  bo.put(0, 1);
  for (int i = 0; i < best_order; ++i) bo.sput(x[i], bps);
  bo.put(0, 2);                // RICE (4-bit parameters)
  bo.put(best_po, 4);
  const int np = 1 << best_po, ps = n >> best_po;
  size_t at = 0;
  for (int pi = 0; pi < np; ++pi) {
    const int cnt = pi == 0 ? ps - best_order : ps;
    const int k = best_k[pi];
    bo.put(k, 4);
    for (int i = 0; i < cnt; ++i) {
      const uint32_t v = best_u[at + i];
      bo.unary(v >> k);
      bo.put(v & ((1u << k) - 1), k);
    }
    at += cnt;
  }
}

void put_utf8(BitOut& bo, uint64_t v) {   // FLAC's UTF-8-style frame number
  if (v < 0x80) {
    bo.put(v, 8);
    return;
  }
  int nbytes = 2;
  while (nbytes < 7 && v >= (1ull << (5 * nbytes + 1))) ++nbytes;
  const int lead_bits = 7 - nbytes;
  bo.put(((0xffu << (8 - nbytes)) & 0xff) | (v >> (6 * (nbytes - 1))), 8);
  (void)lead_bits;
  for (int i = nbytes - 2; i >= 0; --i) bo.put(0x80 | ((v >> (6 * i)) & 0x3f), 8);
}

}  // namespace

extern "C" size_t ainp_flac_encode_bound(int64_t frames, int channels, int bits_per_sample) {
  if (frames < 0 || channels < 1 || bits_per_sample < 1) return 0;
  const int64_t nblocks = frames / 4096 + 1;
  // verbatim worst case + headers
  return (size_t)(42 + nblocks * (32 + channels * 8) +
                  frames * channels * ((bits_per_sample + 7) / 8 + 1));
}

extern "C" int ainp_flac_encode(const int32_t* samples, int64_t frames, int channels,
                                int bits_per_sample, int sample_rate, uint8_t* out, size_t cap,
                                size_t* out_len) {
  if ((!samples && frames) || frames < 0 || channels < 1 || channels > 8 || !out || !out_len ||
      (bits_per_sample != 8 && bits_per_sample != 16 && bits_per_sample != 24) ||
      sample_rate < 1 || sample_rate > 655350 || frames >= (1ll << 36))
    return fail("ainp_flac_encode: bad argument");
  const int B = 4096;
  const int64_t lo = -(1ll << (bits_per_sample - 1)), hi = (1ll << (bits_per_sample - 1)) - 1;
  for (int64_t i = 0; i < frames * channels; ++i)
    if (samples[i] < lo || samples[i] > hi) return fail("ainp_flac_encode: sample out of range");
  BitOut bo;
  bo.buf.reserve(cap);
  // 'fLaC' + STREAMINFO (last metadata block)
  bo.put(0x664C6143u, 32);
  bo.put(1, 1);
  bo.put(0, 7);
  bo.put(34, 24);
  const int last = (int)(frames % B);
  const int minb = frames == 0 ? B : (frames < B ? (int)frames : (last ? (B < last ? B : B) : B));
  bo.put(frames <= B ? (uint32_t)(frames ? frames : 16) : (uint32_t)B, 16);   // min block
  (void)minb;
  bo.put(frames < B ? (uint32_t)(frames ? frames : 16) : (uint32_t)B, 16);    // max block
  bo.put(0, 24);   // min frame size unknown
  bo.put(0, 24);   // max frame size unknown
  bo.put(sample_rate, 20);
  bo.put(channels - 1, 3);
  bo.put(bits_per_sample - 1, 5);
  bo.put((uint64_t)frames >> 32, 4);
  bo.put((uint64_t)frames & 0xffffffffu, 32);
  const size_t md5_at = bo.buf.size();
  for (int i = 0; i < 4; ++i) bo.put(0, 32);   // MD5, filled below
  Md5 md5;
  const int bytes = (bits_per_sample + 7) / 8;
  std::vector<int32_t> ch(B);
  int64_t fno = 0;
  for (int64_t f0 = 0; f0 < frames; f0 += B, ++fno) {
    const int n = (int)((frames - f0) < B ? (frames - f0) : B);
    const size_t hdr_at = bo.buf.size();
    bo.put(0x3ffe, 14);   // sync
    bo.put(0, 1);
    bo.put(0, 1);         // fixed block size
    bo.put(n == B ? 12 : 7, 4);   // 4096, or 16-bit (n-1) at the end of the header
    bo.put(0, 4);         // sample rate from STREAMINFO
    bo.put(channels - 1, 4);   // independent channels
    bo.put(bits_per_sample == 8 ? 1 : bits_per_sample == 16 ? 4 : 6, 3);
    bo.put(0, 1);
    put_utf8(bo, (uint64_t)fno);
    if (n != B) bo.put(n - 1, 16);
    bo.put(crc8(bo.buf.data() + hdr_at, bo.buf.size() - hdr_at), 8);
    for (int c = 0; c < channels; ++c) {
      for (int i = 0; i < n; ++i) ch[i] = samples[(f0 + i) * channels + c];
      write_subframe(bo, ch.data(), n, bits_per_sample);
    }
    bo.align();
    bo.put(crc16(bo.buf.data() + hdr_at, bo.buf.size() - hdr_at), 16);
    for (int i = 0; i < n; ++i)
      for (int c = 0; c < channels; ++c) {
        const int32_t v = samples[(f0 + i) * channels + c];
        uint8_t le[4];
        for (int b = 0; b < bytes; ++b) le[b] = (uint8_t)((uint32_t)v >> (8 * b));
        md5.update(le, bytes);
      }
  }
  uint8_t dig[16];
  md5.final(dig);
  memcpy(bo.buf.data() + md5_at, dig, 16);
  if (bo.buf.size() > cap) return fail("ainp_flac_encode: output buffer too small");
  memcpy(out, bo.buf.data(), bo.buf.size());
  *out_len = bo.buf.size();
  return AINP_OK;
}
