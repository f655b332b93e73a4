"""Synthetic workloads of BASELINE.json, made by the device generator
(avr_synthesize_stream).  No GPU-independent data exists for them: the reference's own file
(data/GOPR4542.MP4) is absent, so these seeded streams stand in, as SURVEY.md 8d specifies.

  clip(ctx)        configs[1]: 1080p High 4:2:0, 64 frames x 1 slice, GOP I + 31 P (twice), QP 26
  corpus(ctx)      configs[4]: mixed I/P/B GOPs, 1/2/4/8/17 slices per frame, 720p/1080p/4K,
                   progressive plus two 1080i streams (field pictures and MBAFF), plus the two real
                   fixtures (tests/fixtures)
  stream_4k(ctx)   configs[3]: one 4K stream, 1 slice per frame, 1-s GOP (I + 29 P) tiled with
                   rewritten frame numbers (avr_synthesize_stream's repeat)
  mixed_files(ctx) many independent files of mixed kinds and sizes: the corpus entries with a seed
                   and a length of their own each (plus the fixtures), for the reference model's
                   files-in-parallel leg
"""
from __future__ import annotations

from pathlib import Path

from . import SynthParams

ROOT = Path(__file__).resolve().parents[1]
FIXTURES = ("realshort.mp4", "cockatoo.mp4")


def clip(ctx, frames: int = 64, mb_width: int = 120, mb_height: int = 68, seed: int = 0) -> bytes:
    return ctx.synthesize(SynthParams(mb_width=mb_width, mb_height=mb_height, slice_type=0, slice_qp=26,
                                      chroma_format_idc=1, transform_8x8_mode=1, seed=seed, gop_length=32), frames)


# (name, mb_width, mb_height, slices per picture, frames, gop, slice type between I pictures, QP,
#  chroma, structure: 0 progressive, 1 field pictures (two fields per frame), 2 MBAFF)
CORPUS = [
    ("720p_IBBP_2spf", 80, 45, 2, 24, 12, 1, 24, 1, 0),
    ("720p_IP_1spf", 80, 45, 1, 32, 16, 0, 28, 1, 0),
    ("1080p_IBBP_4spf", 120, 68, 4, 16, 8, 1, 26, 1, 0),
    ("1080p_IP_17spf", 120, 68, 17, 8, 8, 0, 22, 1, 0),
    ("1080p_I_8spf_422", 120, 68, 8, 4, 1, 2, 30, 2, 0),
    ("4K_IP_8spf", 240, 135, 8, 6, 6, 0, 27, 1, 0),
    ("4K_IBBP_1spf_444", 240, 135, 1, 4, 4, 1, 30, 3, 0),
    ("1080i_PAFF_IP_2spf", 120, 68, 2, 8, 8, 0, 26, 1, 1),
    ("1080i_MBAFF_IBBP_2spf", 120, 68, 2, 8, 8, 1, 26, 1, 2),
]


def slices_of(entry, frames: int) -> int:
    """Slices the generator writes for `frames` frames of a CORPUS entry."""
    spf, structure = entry[3], entry[9]
    return frames * spf * (2 if structure == 1 else 1)


def corpus(ctx, scale: float = 1.0, fixtures: bool = True) -> list[tuple[str, bytes]]:
    """configs[4]: [(name, file bytes)].  scale < 1 shortens every stream (tests)."""
    out = []
    for k, (name, w, h, spf, frames, gop, st, qp, cf, structure) in enumerate(CORPUS):
        n = max(1, int(round(frames * scale)))
        p = SynthParams(mb_width=w, mb_height=h, slice_type=st, slice_qp=qp, chroma_format_idc=cf,
                        transform_8x8_mode=1, num_ref_idx_l0=2, num_ref_idx_l1=1, seed=4000 + k,
                        slices_per_picture=spf, gop_length=gop, structure=structure)
        out.append((name, ctx.synthesize(p, n)))
    if fixtures:
        for f in FIXTURES:
            out.append((f, (ROOT / "tests" / "fixtures" / f).read_bytes()))
    return out


def stream_4k(ctx, seconds: int = 600, fps: int = 30, mb_width: int = 240, mb_height: int = 135,
              seed: int = 0) -> bytes:
    """configs[3]: `seconds` of 4K at `fps`, one slice per frame: one 1-s GOP (I + fps-1 P, QP 26)
    generated once and tiled `seconds` times with rewritten frame_num / idr_pic_id."""
    p = SynthParams(mb_width=mb_width, mb_height=mb_height, slice_type=0, slice_qp=26, chroma_format_idc=1,
                    transform_8x8_mode=1, seed=seed, gop_length=fps, repeat=seconds)
    return ctx.synthesize(p, fps)


def mixed_files(ctx, n: int = 256, scale: float = 0.25, seed: int = 5000) -> list[tuple[str, bytes]]:
    """n independent files cycling through the CORPUS kinds (and, every 16th, a fixture), each with
    its own seed and a frame count drawn from 1 .. 2 x the kind's scaled length, so sizes and
    slice structures differ from file to file (a heterogeneous load, not n copies of one file)."""
    import random
    rnd = random.Random(seed)
    fixtures = [(f, (ROOT / "tests" / "fixtures" / f).read_bytes()) for f in FIXTURES]
    out = []
    for i in range(n):
        if i % 16 == 15:
            out.append(fixtures[(i // 16) % len(fixtures)])
            continue
        name, w, h, spf, frames, gop, st, qp, cf, structure = CORPUS[i % len(CORPUS)]
        nf = max(1, rnd.randint(1, max(1, int(round(2 * frames * scale)))))
        p = SynthParams(mb_width=w, mb_height=h, slice_type=st, slice_qp=qp + rnd.randint(-2, 2), chroma_format_idc=cf,
                        transform_8x8_mode=1, num_ref_idx_l0=2, num_ref_idx_l1=1, seed=seed + i,
                        slices_per_picture=spf, gop_length=gop, structure=structure)
        out.append((f"{name}_{nf}f_s{seed + i}", ctx.synthesize(p, nf)))
    return out
