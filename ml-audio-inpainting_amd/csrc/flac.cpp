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
        case 2: pred = 2 * out[i - 1] - out[i - 2]; break;
        case 3: pred = 3 * out[i - 1] - 3 * out[i - 2] + out[i - 3]; break;
        case 4: pred = 4 * out[i - 1] - 6 * out[i - 2] + 4 * out[i - 3] - out[i - 4]; break;
        default: break;
      }
      out[i] += pred;
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
      for (int j = 0; j < order; ++j) sum += coef[j] * out[i - 1 - j];
      out[i] += sum >> shift;
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
      for (int i = 0; i < blocksize; ++i) ch[1][i] = ch[0][i] - ch[1][i];
    } else if (ch_code == 9) {
      for (int i = 0; i < blocksize; ++i) ch[0][i] += ch[1][i];
    } else if (ch_code == 10) {
      for (int i = 0; i < blocksize; ++i) {
        const int64_t side = ch[1][i];
        const int64_t mid = (ch[0][i] * 2) | (side & 1);
        ch[0][i] = (mid + side) >> 1;
        ch[1][i] = (mid - side) >> 1;
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
