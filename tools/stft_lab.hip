// stft_lab.hip — timing lab for the fused n_fft=512 STFT/feature kernel on
// the C2 batch (32 x 4 s clips, hop 192, win 384, T=334, 3200-sample gaps).
// Builds standalone against the product source (no libainp.so):
//   hipcc -O3 -std=c++17 --offload-arch=gfx950 tools/stft_lab.hip -o tools/stft_lab
// Prints us/launch and algorithmic GB/s (4880 B/frame) per variant, and compares
// candidate kernels' outputs with the product kernel's (tools/stft512b.inc:
// b = the staged kernel now in the product, c = unstaged direct stores,
// d = two alternating teams per workgroup; build with -DSTFTB_OCC=2
// -DSTFTC_OCC=2 -DSTFTB_PASSA=1 -DSTFTB_J0=1).
// Measured on MI355X (C2 batch, 52.2 MB/launch): round-1 kernel 29.9 us; its
// FFT-only / store-only probes 22.2 / 12.9 us (base 5 us) -- no overlap;
// b 24.2 us (grid 512), c 23.5 us (stores uncoalesced: 13 us of its 27),
// d 26.5 us.  fp64 issue rate: tools/fp64_rate.hip.
#include "../ml-audio-inpainting_amd/csrc/stft.hip"
#include "stft512b.inc"

#include <math.h>
#include <stdio.h>
#include <string.h>
#include <vector>

namespace ainp {
int record_error(hipError_t e, const char* where) {
  fprintf(stderr, "%s: %s\n", where, hipGetErrorString(e));
  return -1;
}
int record_msg(const char* msg) {
  fprintf(stderr, "%s\n", msg);
  return -1;
}
}  // namespace ainp

#define CK(x)                                                                   \
  do {                                                                          \
    hipError_t e_ = (x);                                                        \
    if (e_ != hipSuccess) {                                                     \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
      exit(1);                                                                  \
    }                                                                           \
  } while (0)

static const int B = 32, S = 64000, HOP = 192, NFFT = 512, WIN = 384, T = 334, GAP = 3200;

struct Bufs {
  float *audio, *o0, *o1, *o2;
  int64_t* gs;
  double* win;
};

template <typename L>
static double time_us(L launch, int reps = 50) {
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  for (int i = 0; i < 5; ++i) launch();
  CK(hipDeviceSynchronize());
  CK(hipEventRecord(a));
  for (int i = 0; i < reps; ++i) launch();
  CK(hipEventRecord(b));
  CK(hipEventSynchronize(b));
  float ms;
  CK(hipEventElapsedTime(&ms, a, b));
  return ms * 1e3 / reps;
}

static void report(const char* name, double us) {
  const double bytes = 4880.0 * B * T;
  printf("%-44s %8.2f us  %7.1f GB/s  frac %.3f\n", name, us, bytes / us / 1e3,
         bytes / us / 1e3 / 8000.0);
  fflush(stdout);
}

static void launch_prod(const Bufs& d, int64_t grid) {
  const int64_t ntt = (T + f512::TF - 1) / f512::TF;
  hipLaunchKernelGGL((f512::stft512_kernel<AINP_FEAT_CNNBLSTM, true>), dim3(grid),
                     dim3(f512::NT), f512::LDS_BYTES, 0, d.audio, (int64_t)S, nullptr, d.gs,
                     (int64_t)B, (int64_t)GAP, (int64_t)16000, d.win, HOP, (int64_t)T, ntt,
                     d.o0, d.o1, d.o2, nullptr);
}

static void launch_b(const Bufs& d, int64_t grid) {
  const int64_t ntt = (T + f512::TF - 1) / f512::TF;
  hipLaunchKernelGGL((f512b::stft512b_kernel<AINP_FEAT_CNNBLSTM, true>), dim3(grid),
                     dim3(f512::NT), f512b::LDS_BYTES, 0, d.audio, (int64_t)S, nullptr, d.gs,
                     (int64_t)B, (int64_t)GAP, (int64_t)16000, d.win, HOP, (int64_t)T, ntt,
                     d.o0, d.o1, d.o2, nullptr);
}

static void launch_c(const Bufs& d, int64_t grid) {
  hipLaunchKernelGGL((f512c::stft512c_kernel<AINP_FEAT_CNNBLSTM, true>), dim3(grid),
                     dim3(f512c::NT), f512c::LDS_BYTES, 0, d.audio, (int64_t)S, nullptr, d.gs,
                     (int64_t)B, (int64_t)GAP, (int64_t)16000, d.win, HOP, (int64_t)T,
                     d.o0, d.o1, d.o2, nullptr);
}

static void launch_d(const Bufs& d, int64_t grid) {
  const int64_t ntt = (T + f512::TF - 1) / f512::TF;
  hipLaunchKernelGGL((f512d::stft512d_kernel<AINP_FEAT_CNNBLSTM, true>), dim3(grid),
                     dim3(f512d::NTD), f512d::LDS_BYTES, 0, d.audio, (int64_t)S, nullptr, d.gs,
                     (int64_t)B, (int64_t)GAP, (int64_t)16000, d.win, HOP, (int64_t)T, ntt,
                     d.o0, d.o1, d.o2, nullptr);
}

static void compare(const char* nm, const std::vector<float>& a, const std::vector<float>& b) {
  double mx = 0, mref = 0;
  size_t ndiff = 0, nbad = 0;
  for (size_t i = 0; i < a.size(); ++i) {
    const double e = fabs((double)a[i] - (double)b[i]);
    if (a[i] != b[i]) ++ndiff;
    if (!(e <= 1e-5 * (1.0 + fabs((double)a[i])))) ++nbad;
    if (e > mx || e != e) mx = e;
    mref = fmax(mref, fabs((double)a[i]));
  }
  printf("  %-8s max|d| %.3e (max|ref| %.3e)  differing %zu / %zu  beyond 1e-5 rel: %zu\n", nm,
         mx, mref, ndiff, a.size(), nbad);
}

static void fetch(const Bufs& d, size_t plane, std::vector<float>& a, std::vector<float>& b,
                  std::vector<float>& c) {
  a.resize(plane);
  b.resize(2 * plane);
  c.resize(plane);
  CK(hipDeviceSynchronize());
  CK(hipMemcpy(a.data(), d.o0, plane * 4, hipMemcpyDeviceToHost));
  CK(hipMemcpy(b.data(), d.o1, plane * 8, hipMemcpyDeviceToHost));
  CK(hipMemcpy(c.data(), d.o2, plane * 4, hipMemcpyDeviceToHost));
}

int main(int argc, char** argv) {
  const bool only_b = argc > 1 && argv[1][0] == 'b';  // counter runs: the candidate alone
  Bufs d;
  const size_t plane = (size_t)B * 257 * T;
  std::vector<float> ha((size_t)B * S);
  uint32_t st = 12345u;
  for (auto& v : ha) {
    st = st * 1664525u + 1013904223u;
    v = ((st >> 8) * (1.0f / 16777216.0f) - 0.5f) * 0.2f;
  }
  std::vector<int64_t> hg(B);
  for (int i = 0; i < B; ++i) hg[i] = (int64_t)((i * 7919) % (S - GAP));
  std::vector<double> hw(NFFT, 0.0);
  for (int n = 0; n < WIN; ++n) hw[(NFFT - WIN) / 2 + n] = 0.5 - 0.5 * cos(2.0 * M_PI * n / WIN);
  CK(hipMalloc(&d.audio, ha.size() * 4));
  CK(hipMalloc(&d.gs, B * 8));
  CK(hipMalloc(&d.win, NFFT * 8));
  CK(hipMalloc(&d.o0, plane * 4));
  CK(hipMalloc(&d.o1, plane * 8));
  CK(hipMalloc(&d.o2, plane * 4));
  CK(hipMemcpy(d.audio, ha.data(), ha.size() * 4, hipMemcpyHostToDevice));
  CK(hipMemcpy(d.gs, hg.data(), B * 8, hipMemcpyHostToDevice));
  CK(hipMemcpy(d.win, hw.data(), NFFT * 8, hipMemcpyHostToDevice));

  const int64_t ntiles = (int64_t)B * ((T + f512::TF - 1) / f512::TF);
  char nm[96];
  if (only_b) {
    for (int i = 0; i < 6; ++i) {
      if (argv[1][1] == 'c') launch_c(d, atoi(argv[2]));
      else if (argv[1][1] == 'd') launch_d(d, atoi(argv[2]));
      else launch_b(d, ntiles);
    }
    CK(hipDeviceSynchronize());
    printf("done\n");
    return 0;
  }
  report("product (one tile per workgroup)", time_us([&] { launch_prod(d, ntiles); }));
  for (int64_t g : {512, 384, 256}) {
    snprintf(nm, sizeof nm, "product grid %ld", (long)g);
    report(nm, time_us([&] { launch_prod(d, g); }));
  }
  std::vector<float> r0, r1, r2, c0, c1, c2;
  CK(hipMemset(d.o0, 0x7f, plane * 4));
  CK(hipMemset(d.o1, 0x7f, plane * 8));
  CK(hipMemset(d.o2, 0x7f, plane * 4));
  launch_prod(d, ntiles);
  fetch(d, plane, r0, r1, r2);
  CK(hipMemset(d.o0, 0x7f, plane * 4));
  CK(hipMemset(d.o1, 0x7f, plane * 8));
  CK(hipMemset(d.o2, 0x7f, plane * 4));
  launch_b(d, ntiles);
  fetch(d, plane, c0, c1, c2);
  printf("f512b vs product:\n");
  compare("logmag", r0, c0);
  compare("target", r1, c1);
  compare("mask", r2, c2);
  CK(hipMemset(d.o0, 0x7f, plane * 4));
  CK(hipMemset(d.o1, 0x7f, plane * 8));
  CK(hipMemset(d.o2, 0x7f, plane * 4));
  launch_c(d, 256);
  fetch(d, plane, c0, c1, c2);
  printf("f512c vs product:\n");
  compare("logmag", r0, c0);
  compare("target", r1, c1);
  compare("mask", r2, c2);
  for (int64_t g : {256, 512, 768}) {
    snprintf(nm, sizeof nm, "f512c grid %ld", (long)g);
    report(nm, time_us([&] { launch_c(d, g); }));
  }
  CK(hipMemset(d.o0, 0x7f, plane * 4));
  CK(hipMemset(d.o1, 0x7f, plane * 8));
  CK(hipMemset(d.o2, 0x7f, plane * 4));
  launch_d(d, 256);
  fetch(d, plane, c0, c1, c2);
  printf("f512d vs product:\n");
  compare("logmag", r0, c0);
  compare("target", r1, c1);
  compare("mask", r2, c2);
  for (int64_t g : {224, 256, 336}) {
    snprintf(nm, sizeof nm, "f512d grid %ld", (long)g);
    report(nm, time_us([&] { launch_d(d, g); }));
  }
  report("f512b (one tile per workgroup)", time_us([&] { launch_b(d, ntiles); }));
  for (int64_t g : {768, 512}) {
    snprintf(nm, sizeof nm, "f512b grid %ld", (long)g);
    report(nm, time_us([&] { launch_b(d, g); }));
  }
  CK(hipDeviceSynchronize());
  printf("done\n");
  return 0;
}
