"""MI355X-native speaker-embedding extractor (the tf_extract.py hot path of
xx205/voxsrc2020_speaker_verification), built on hand-written gfx950 HIP kernels
behind a C-ABI (`include/voxemb.h`)."""

__version__ = "0.1.0"
