"""oracle/ -- TEST INFRASTRUCTURE ONLY.

CPU restatements of the reference's hot-path algorithms
(savage-hacker14/ml-audio-inpainting), used exclusively as the checker by
tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg.  Nothing in
the product package (ml-audio-inpainting_amd/) imports this package; the
product path runs only the HIP kernels of libainp.so and fails loudly when
they are missing.

Pinning (see DESIGN.md "Oracle"):
  * stft_ref / features: librosa>=0.10 stft semantics restated in numpy
    float64 (librosa is not installed here, so exact librosa output is
    "parity unpinned"; the restatement is checked against numpy's own FFT,
    against the reference tests' properties (F = n_fft/2+1, frame counts,
    STFT->ISTFT identity) and against committed known-answer gap indices).
  * cnnblstm_ref: torch-CPU restatement of StackedBLSTMCNN + the training
    step, pinned by golden vectors produced by importing the reference's own
    models/CNNBLSTM/model.py (tests/golden/gen_golden.py).
"""
