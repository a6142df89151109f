"""Drop-in for models/model_eval.py: inpaint the test_samples
clips with a fixed 80 ms gap at 2.0 s and write the reconstructed audio.

Follows models/model_eval.py:23-227 step by step, on the MI355X kernels:
  load_model      (:23-46)  PConvUNet / StackedBLSTMCNN from a state_dict
                            (loaded with weights_only=True, not False), eval()
  inpaint         (:48-195) load_audio -> create_gap_mask(0.08 s at 2.0 s) ->
                            extract_spectrogram of the clean and gapped audio
                            (GPU STFT) ->
      gan:      log1p magnitudes, frame mask [s//hop, ceil(e/hop)) of 1=valid,
                G(impaired, mask) -> spectrogram_to_audio(output, phase=original
                phase) -- the generator's log1p-domain output goes to the ISTFT
                as the magnitude, as the reference passes it (:162-173);
      cnnlstm:  mask [time_to_frames(2.0), time_to_frames(2.08)) of 1=gap,
                log10(|X (1 - mask)| + 1e-9) of the ORIGINAL spectrogram,
                10 ** model.reconstruct_spectrogram(...) ->
                spectrogram_to_audio(..., phase=original phase) (:174-191);
                    -> save_audio (peak-normalised FLAC, native encoder)
  run_evaluation  (:198-227) every .flac of input_dir -> <name>_<type>_inpainted.flac
Spectrogram plots (:157-162,180-185) are out of scope (plotting).  The ISTFT
runs on the GPU (ainp_istft); output length hop * (T - 1), as librosa's.
"""
from __future__ import annotations

import os
import sys

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
_PKG = os.path.dirname(HERE)
for _p in (HERE, _PKG):
    if _p not in sys.path:
        sys.path.insert(0, _p)

import utils  # noqa: E402
from models.CNNBLSTM.model import StackedBLSTMCNN  # noqa: E402
from models.GAN.networks import PConvUNet  # noqa: E402

GAP_LEN_S = 0.08      # model_eval.py:64
GAP_START_S = 2.0     # model_eval.py:70

DEFAULT_ENC = [(64, 7, 2, 3), (128, 5, 2, 2), (256, 5, 2, 2),
               (512, 3, 2, 1), (512, 3, 2, 1), (512, 3, 2, 1), (512, 3, 2, 1)]


def load_config(config_path):
    import yaml
    with open(config_path, "r") as f:
        return yaml.safe_load(f)


def load_model(model_type, config_path, checkpoint_path, device):
    """model_eval.py:23-46."""
    print(f"Loading {model_type} model from {checkpoint_path}...")
    if model_type == "gan":
        cfg = load_config(config_path)
        g = cfg["model"]["generator"]
        model = PConvUNet(input_channels=g["input_channels"], mask_channels=g["mask_channels"],
                          output_channels=g["output_channels"],
                          enc_layer_cfg=g.get("enc_layer_cfg", DEFAULT_ENC)).to(device)
    elif model_type == "cnnlstm":
        model = StackedBLSTMCNN(config_path).to(device)
    else:
        raise ValueError(f"Unknown model type: {model_type}")
    sd = checkpoint_path if isinstance(checkpoint_path, dict) else \
        torch.load(checkpoint_path, weights_only=True, map_location=device)
    model.load_state_dict(sd)
    model.eval()
    return model


def _time_to_frames(t, sr, hop):
    """librosa.time_to_frames."""
    return int(np.asarray(t * sr).astype(int)) // hop


def inpaint(model, config_path, audio_path, output_path, device):
    """model_eval.py:48-195; returns the reconstructed audio (also written)."""
    if isinstance(model, PConvUNet):
        model_type = "gan"
    elif isinstance(model, StackedBLSTMCNN):
        model_type = "cnnlstm"
    else:
        raise ValueError("Unknown model type.")
    config = load_config(config_path)
    sp = config["data"]["spectrogram"]
    n_fft, hop, win = sp["n_fft"], sp["hop_length"], sp["win_length"]

    audio, sr = utils.load_audio(audio_path)
    mask_td, (gap_start_sample, gap_end_sample) = utils.create_gap_mask(
        len(audio), GAP_LEN_S, sr, gap_start_s=GAP_START_S)
    impaired_audio = audio * mask_td
    original_spectrogram = utils.extract_spectrogram(audio, n_fft=n_fft, hop_length=hop,
                                                     win_length=win)
    original_magnitude = np.log1p(np.abs(original_spectrogram))
    original_phase = np.angle(original_spectrogram)

    if model_type == "gan":
        impaired_spectrogram = utils.extract_spectrogram(impaired_audio, n_fft=n_fft,
                                                         hop_length=hop, win_length=win)
        impaired_magnitude = np.log1p(np.abs(impaired_spectrogram))
        gs = gap_start_sample // hop
        ge = int(np.ceil(gap_end_sample / hop))
        T = original_magnitude.shape[1]
        gs, ge = max(0, gs), min(T, ge)
        spec_mask = np.ones_like(original_magnitude, dtype=np.float32)
        if ge > gs:
            spec_mask[:, gs:ge] = 0
        imp_t = torch.from_numpy(impaired_magnitude.astype(np.float32)).to(device)[None, None]
        mask_t = torch.from_numpy(spec_mask).to(device)[None, None]
        with torch.no_grad():
            inpainted = model(imp_t, mask_t)[0, 0]
    else:
        spec_mask = np.zeros(original_spectrogram.shape, dtype=np.float32)
        fs = _time_to_frames(GAP_START_S, sr, hop)
        fe = _time_to_frames(2.08, sr, hop)           # model_eval.py:149
        spec_mask[:, fs:fe] = 1
        mask_t = torch.from_numpy(spec_mask).to(device)
        log_imp = np.log10(np.abs(original_spectrogram * (1 - spec_mask)) + 1e-9)
        log_imp_t = torch.from_numpy(log_imp.astype(np.float32))[None].to(device)
        with torch.no_grad():
            inpainted = (10 ** model.reconstruct_spectrogram(log_imp_t, mask_t))[0]
    y = utils.spectrogram_to_audio(inpainted.float().cpu().numpy(), phase=original_phase,
                                   phase_info=False, n_fft=n_fft, hop_length=hop,
                                   win_length=win)
    utils.save_audio(y, file_path=output_path, sample_rate=sr)
    return y


def run_evaluation(input_dir, output_dir, model_type, checkpoint, config_path):
    """model_eval.py:198-227."""
    if not os.path.isdir(input_dir):
        print(f"Error: Input directory not found: {input_dir}")
        return
    if not isinstance(checkpoint, dict) and not os.path.exists(checkpoint):
        print(f"Error: Checkpoint file not found: {checkpoint}")
        return
    os.makedirs(output_dir, exist_ok=True)
    if not torch.cuda.is_available():
        raise RuntimeError("model_eval runs on the MI355X kernels: no GPU visible")
    device = torch.device("cuda")
    model = load_model(model_type, config_path, checkpoint, device)
    flac_files = sorted(f for f in os.listdir(input_dir) if f.lower().endswith(".flac"))
    print(f"Found {len(flac_files)} .flac files in {input_dir}")
    outs = []
    for filename in flac_files:
        out = os.path.join(output_dir, f"{os.path.splitext(filename)[0]}_{model_type}_inpainted.flac")
        inpaint(model, config_path, os.path.join(input_dir, filename), out, device)
        outs.append(out)
    return outs


if __name__ == "__main__":
    # model_eval.py:229-256 (CNN-LSTM configuration by default)
    run_evaluation(input_dir=sys.argv[1] if len(sys.argv) > 1 else "../test_samples",
                   output_dir=sys.argv[2] if len(sys.argv) > 2 else "../test_samples_reconstructed",
                   model_type=sys.argv[3] if len(sys.argv) > 3 else "cnnlstm",
                   checkpoint=sys.argv[4] if len(sys.argv) > 4 else
                   "CNNBLSTM/checkpoints/blstm_cnn_epoch_75.pt",
                   config_path=sys.argv[5] if len(sys.argv) > 5 else "CNNBLSTM/cnn_blstm.yaml")
