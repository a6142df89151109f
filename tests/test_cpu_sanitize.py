"""Host sanitizer runs (SURVEY §5 "race detection / sanitizers"; VERDICT r02
item 9).  GPU AddressSanitizer is not available for gfx950 on this pool, so
the host C++ that parses untrusted input runs under ASan + UBSan on the CPU:

  csrc/flac.cpp (the FLAC bitstream decoder / encoder that replaces soundfile
  behind utils.load_audio / save_audio, /root/reference/utils.py:36,87):
  every bundled LibriSpeech clip decoded whole, 20 truncations and 240
  seeded corruptions each, and encoder round trips (8/16/24-bit, mono and
  stereo, ragged last blocks) -- tests/sanitize/flac_fuzz.cpp.

The torch.ops.ainp host layer (csrc/torch_ops.cpp) is built with UBSan as
libainp_torch_ubsan.so; test_gpu_sanitize.py runs it on the GPU box."""
import glob
import os
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, "ml-audio-inpainting_amd", "csrc")


@pytest.fixture(scope="module")
def sanitize_build():
    r = subprocess.run(["make", "-C", CSRC, "sanitize"], capture_output=True, text=True,
                       timeout=900)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-2000:]
    return os.path.join(CSRC, "build", "flac_fuzz")


@pytest.mark.timeout(900)
def test_flac_codec_under_asan_ubsan(sanitize_build):
    clips = sorted(glob.glob(os.path.join(ROOT, "tests", "golden", "flac", "*.flac")))
    assert len(clips) == 9
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:halt_on_error=1:abort_on_error=0",
               UBSAN_OPTIONS="halt_on_error=1:print_stacktrace=1")
    r = subprocess.run([sanitize_build] + clips, capture_output=True, text=True, timeout=800,
                       env=env)
    out = r.stdout + r.stderr
    assert r.returncode == 0, out[-3000:]
    assert "flac_fuzz OK" in out
    assert "runtime error" not in out and "AddressSanitizer" not in out, out[-3000:]
    assert out.count("mutated decodes") == 9


def test_torch_ops_ubsan_library_built(sanitize_build):
    so = os.path.join(ROOT, "ml-audio-inpainting_amd", "ainp", "libainp_torch_ubsan.so")
    assert os.path.exists(so)
    r = subprocess.run(["readelf", "-d", so], capture_output=True, text=True)
    assert "libubsan" in r.stdout
