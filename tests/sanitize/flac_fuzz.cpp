// flac_fuzz.cpp -- host sanitizer harness for csrc/flac.cpp (the FLAC
// bitstream decoder / encoder behind utils.load_audio / save_audio, replacing
// soundfile at /root/reference/utils.py:36,87).  Built with
// -fsanitize=address,undefined by `make -C ml-audio-inpainting_amd/csrc
// sanitize` and run by tests/test_cpu_sanitize.py:
//
//   flac_fuzz <file.flac>...   decode each file (whole), then every prefix
//                              truncation at 20 lengths and 240 seeded
//                              single-bit / single-byte corruptions: the
//                              decoder must return an error or decode, never
//                              touch memory outside its buffers;
//   (always)                   encoder round trips on seeded PCM (8/16/24-bit,
//                              1-2 channels, silence, full scale, ragged
//                              final blocks) decoded back bit-exactly.
// Exit 0 when everything held; any sanitizer report aborts (halt_on_error).
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <vector>

#include "../../include/ainp.h"

namespace ainp {
int record_msg(const char*) { return AINP_EINVAL; }
}

static uint64_t rng_state = 0x9e3779b97f4a7c15ull;
static uint32_t rnd() {
  rng_state ^= rng_state << 13;
  rng_state ^= rng_state >> 7;
  rng_state ^= rng_state << 17;
  return (uint32_t)(rng_state >> 11);
}

static int decode_all(const std::vector<uint8_t>& d, std::vector<int32_t>& out, int64_t* nf) {
  int sr = 0, ch = 0, bps = 0;
  int64_t frames = 0;
  uint8_t md5[16];
  if (ainp_flac_info(d.data(), d.size(), &sr, &ch, &bps, &frames, md5) != 0) return -1;
  if (ch < 1 || ch > 8 || frames < 0 || frames > (int64_t)1 << 22) return -1;
  out.assign((size_t)(frames ? frames : 1) * ch, 0);
  return ainp_flac_decode(d.data(), d.size(), out.data(), frames, nf);
}

static int fuzz_file(const char* path) {
  FILE* f = fopen(path, "rb");
  if (!f) { fprintf(stderr, "cannot open %s\n", path); return 1; }
  std::vector<uint8_t> d;
  uint8_t buf[65536];
  size_t k;
  while ((k = fread(buf, 1, sizeof buf, f)) > 0) d.insert(d.end(), buf, buf + k);
  fclose(f);
  std::vector<int32_t> ref;
  int64_t nf = 0;
  if (decode_all(d, ref, &nf) != 0) { fprintf(stderr, "decode failed: %s\n", path); return 1; }
  std::vector<int32_t> out;
  int ok = 0, err = 0;
  for (int i = 1; i <= 20; ++i) {       // truncations
    std::vector<uint8_t> t(d.begin(), d.begin() + (size_t)((double)d.size() * i / 21.0));
    int64_t n2 = 0;
    (decode_all(t, out, &n2) == 0 ? ok : err)++;
  }
  for (int i = 0; i < 240; ++i) {       // corruptions (header region weighted)
    std::vector<uint8_t> t = d;
    const size_t at = (i & 1) ? rnd() % (t.size() < 256 ? t.size() : 256) : rnd() % t.size();
    if (i & 2) t[at] ^= (uint8_t)(1u << (rnd() & 7));
    else t[at] = (uint8_t)rnd();
    int64_t n2 = 0;
    (decode_all(t, out, &n2) == 0 ? ok : err)++;
  }
  printf("%s: %lld frames, mutated decodes ok=%d rejected=%d\n", path, (long long)nf, ok, err);
  return 0;
}

static int round_trip(int64_t frames, int channels, int bps, int kind) {
  std::vector<int32_t> pcm((size_t)frames * channels);
  const int32_t hi = (1 << (bps - 1)) - 1, lo = -(1 << (bps - 1));
  for (size_t i = 0; i < pcm.size(); ++i) {
    int32_t v;
    if (kind == 0) v = 0;                                     // silence
    else if (kind == 1) v = (i & 1) ? hi : lo;                // full-scale square
    else if (kind == 2) v = (int32_t)(rnd() % (uint32_t)(hi - lo + 1)) + lo;   // noise
    else v = (int32_t)((double)hi * 0.6 * __builtin_sin(0.01 * (double)(i / channels)));
    pcm[i] = v;
  }
  const size_t cap = ainp_flac_encode_bound(frames, channels, bps);
  std::vector<uint8_t> enc(cap);
  size_t len = 0;
  if (ainp_flac_encode(pcm.data(), frames, channels, bps, 16000, enc.data(), cap, &len) != 0) {
    fprintf(stderr, "encode failed (%lld, %d, %d, %d)\n", (long long)frames, channels, bps, kind);
    return 1;
  }
  enc.resize(len);
  std::vector<int32_t> dec;
  int64_t nf = 0;
  if (decode_all(enc, dec, &nf) != 0 || nf != frames ||
      memcmp(dec.data(), pcm.data(), pcm.size() * sizeof(int32_t)) != 0) {
    fprintf(stderr, "round trip mismatch (%lld, %d, %d, %d)\n", (long long)frames, channels, bps,
            kind);
    return 1;
  }
  return 0;
}

int main(int argc, char** argv) {
  int bad = 0;
  for (int i = 1; i < argc; ++i) bad |= fuzz_file(argv[i]);
  const int64_t lens[] = {1, 15, 16, 4095, 4096, 4097, 12345, 80000};
  for (int64_t n : lens)
    for (int ch = 1; ch <= 2; ++ch)
      for (int bps : {8, 16, 24})
        for (int kind = 0; kind < 4; ++kind) bad |= round_trip(n, ch, bps, kind);
  printf(bad ? "FAILED\n" : "flac_fuzz OK\n");
  return bad;
}
