/*
 * voxemb.h -- C-ABI of libvoxemb.so, the MI355X (gfx950) speaker-embedding
 * extractor that replaces the TF1 frozen-graph forward of
 * xx205/voxsrc2020_speaker_verification's `tensorflow/tf_extract.py`.
 *
 * Plain pointers and sizes only; no torch / HIP types cross the boundary
 * (streams are passed as `void*` = hipStream_t, NULL = the handle's stream).
 * Every function returns VOX_OK (0) or a negative status; the thread-local
 * message is available from vox_last_error().  Ownership: callers own every
 * buffer they pass in; the handle owns its device weights and workspace.
 *
 * Reference interfaces replaced (file:line under the reference repo):
 *   vox_load / vox_load_blob  <- tf.GraphDef().ParseFromString + import_graph_def
 *                                (tensorflow/tf_extract.py:75-82)
 *   vox_dim                   <- width of tensor "model/outputs:0"
 *                                (tensorflow/models/res2net_model.py:242,
 *                                 tdnn_model.py:153, dpn_model.py:168)
 *   vox_embed                 <- sess.run(model/outputs:0, {model/inputs:0: x})
 *                                (tensorflow/tf_extract.py:108); x is the
 *                                [N,T,F] batch before tf_extract's expand_dims
 *                                (tf_extract.py:32)
 *   vox_embed_device          <- same, inputs already resident in HBM
 *   vox_embed_utt             <- the chunk loop + length-weighted average
 *                                (tensorflow/tf_extract.py:96-111)
 *   vox_stats_pool_device     <- stats_pool (tensorflow/models/models.py:262-269)
 *   vox_asnorm_stats          <- get_cohort_mean_std (tensorflow/snorm.py:83-109)
 *                                followed by the head's first BN
 *                                (res2net_model.py:239)
 *   vox_sliding_cmn           <- Kaldi `apply-cmvn-sliding --norm-vars=false
 *                                --center=true --cmn-window=300`
 *                                (tensorflow/tf_extract.py:63)
 *   vox_mat_shape/vox_read_mat<- kaldi_io.read_mat / _read_mat_binary /
 *                                _read_compressed_mat (tensorflow/kaldi_io.py:420-504)
 *   vox_format_vec_flt        <- kaldi_io.write_vec_flt (kaldi_io.py:304-334)
 *                                + `copy-vector ark:- ark,scp:` (tf_extract.py:65)
 */
#ifndef VOXEMB_H
#define VOXEMB_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define VOX_OK 0
#define VOX_EINVAL (-22)   /* bad argument / shape mismatch                 */
#define VOX_ENOMEM (-12)   /* host or device allocation failed              */
#define VOX_EIO (-5)       /* file missing / malformed blob / bad ark       */
#define VOX_ESHORT (-61)   /* utterance shorter than 25 frames: the reference
                              raises ZeroDivisionError (tf_extract.py:102,111) */
#define VOX_EHIP (-1000)   /* HIP runtime error                             */

#define VOX_FP32 0         /* fp32 activations, f32-input MFMA (parity mode) */
#define VOX_BF16 1         /* bf16 activations, bf16 MFMA, fp32 accumulate   */

typedef struct vox_model vox_model;

/* Load a VOXEMB01 weight blob (file or memory) onto HIP device `device`. */
int vox_load(const char* blob_path, int device, int precision, vox_model** out);
int vox_load_blob(const void* blob, size_t nbytes, int device, int precision,
                  vox_model** out);
void vox_free(vox_model* m);

int vox_dim(const vox_model* m);         /* embedding width (256 / 192)      */
int vox_feat_dim(const vox_model* m);    /* expected F (mel bins)            */
int vox_expand_dim(const vox_model* m);  /* 2 = TDNN layout, 3 = 2-D layout  */
int vox_precision(const vox_model* m);

/* x: host [n,t,f] float32 row-major; out: host [n, vox_dim] float32. */
int vox_embed(vox_model* m, const float* x, int n, int t, int f, float* out);
/* d_x, d_out: device pointers on the handle's device; stream may be NULL (the
 * handle's own non-blocking stream -- NOT the HIP default stream: work the
 * caller queued on the default stream is not ordered before it, so pass an
 * explicit stream, or synchronise, when the inputs were produced there). */
int vox_embed_device(vox_model* m, const float* d_x, int n, int t, int f,
                     float* d_out, void* stream);
/* Ragged batches: utterance i of the [n,t,f] batch holds lens[i] frames
 * (1 <= lens[i] <= t), its rows past them are padding (any values).  Each
 * embedding equals the one vox_embed computes for that utterance alone at
 * t = lens[i] (the same per-utterance chunk as tf_extract.py:108 runs), bit for
 * bit: every kernel that reads a row's neighbours treats the padded rows as
 * the SAME / fixed padding of an utterance that ends at lens[i], and the stats
 * pool averages its lens[i] (downsampled) rows.  So chunks of different
 * lengths share one batch and one resident plan keyed on (n, t) -- what the
 * streaming extractor buckets real length distributions into.  res2net models
 * without attentive pooling and tdnn models, VOX_BF16; other plans (dpn68, the
 * attentive models, fp32) return VOX_EINVAL.
 * _device: d_lens is a device int32 [n] array (read in stream order);
 * vox_embed_lens: host buffers, lens checked on the host. */
int vox_embed_device_lens(vox_model* m, const float* d_x, int n, int t, int f,
                          const int* d_lens, float* d_out, void* stream);
int vox_embed_lens(vox_model* m, const float* x, int n, int t, int f, const int* lens,
                   float* out);
/* One utterance of any length t >= 25, chunked at 1000 frames. */
int vox_embed_utt(vox_model* m, const float* x, int t, int f, float* out);

/* Per-op profile of one forward at (n, t): runs the plan `reps` times with
 * HIP events around every op on `stream`.  Fills up to `max_ops` entries:
 * op_ms (average ms per launch), op_flops (algorithmic FLOP per launch),
 * op_bytes (algorithmic HBM bytes per launch), op_kind (0 conv, 1 stats-pool,
 * 2 head, 3 other).  Returns the number of ops (>=0) or a status (<0). */
int vox_profile(vox_model* m, const float* d_x, int n, int t, int f, int reps,
                float* op_ms, double* op_flops, double* op_bytes, int* op_kind,
                int max_ops, void* stream);

/* Text description of the plan at (n, t): one line per kernel launch with
 * its kernel family, tile config, shapes and algorithmic FLOP/bytes.
 * Returns the needed buffer size (bytes incl. NUL) or a status (<0). */
int vox_plan_describe(vox_model* m, const float* d_x, int n, int t, int f, char* buf,
                      size_t cap);

/* Plan residency counters of the handle: plans built (planned + captured),
 * calls served by a resident plan (the current one or a cached one) without
 * re-planning, plans destroyed
 * (evicted, or dropped when the workspace grew), and plans resident now
 * (current + cached; VOXEMB_PLAN_CACHE caps the cached ones, default 64).
 * Any pointer may be NULL. */
int vox_plan_stats(const vox_model* m, int64_t* built, int64_t* hits, int64_t* dropped,
                   int* resident);

/* Standalone stats-pool (+BN) kernel: x NHWC [n,h,w,c] (dtype VOX_FP32 or
 * VOX_BF16), mean/inv per pooled feature (may be NULL = identity),
 * out [n, w*2c] float32 with feature index w*2c + {c | c+C}. */
int vox_stats_pool_device(const void* d_x, int dtype, int n, int h, int w, int c,
                          const float* d_mean, const float* d_inv, float* d_out,
                          void* stream);

/* Adaptive s-norm cohort statistics (tensorflow/snorm.py:83-109,
 * get_cohort_mean_std): for each trial row, the mean and population std of
 * its top-k cosine scores against the cohort rows (callers l2-normalise both,
 * as snorm.py does).  Device pointers: trial [n,d], cohort [m,d] float32,
 * mean/std [n].  k = min(topk, m); d % 4 == 0.  Synchronises `stream`. */
int vox_asnorm_stats(const float* d_trial, int n, const float* d_cohort, int m, int d,
                     int topk, float* d_mean, float* d_std, void* stream);

/* ---- front end on the device: wav -> FBANK -> sliding CMN ---------------
 * Kaldi `compute-fbank-feats` options (conf/fbank80.conf sets only
 * sample_frequency 16000 and num_mel_bins 80; prepare_data.sh:66-70).
 * Fixed as Kaldi's defaults: povey window, snip_edges, padded FFT (256 or 512),
 * no energy term, log power mel energies floored at FLT_EPSILON. */
typedef struct vox_fbank_opts {
  float sample_frequency;         /* 16000 */
  float frame_length_ms;          /* 25 */
  float frame_shift_ms;           /* 10 */
  float dither;                   /* Kaldi default 1.0 (random); 0 = deterministic */
  float preemphasis_coefficient;  /* 0.97 */
  int remove_dc_offset;           /* 1 */
  int num_mel_bins;               /* Kaldi default 23; 80 / 40 in conf/fbank{80,40}.conf */
  float low_freq;                 /* 20 */
  float high_freq;                /* 0: Nyquist (negative: offset from Nyquist) */
  uint64_t seed;                  /* dither noise = f(seed, utterance key, frame, sample) */
} vox_fbank_opts;
void vox_fbank_default_opts(vox_fbank_opts* o);
/* Frames of an utterance of num_samples samples (snip_edges), or < 0. */
int64_t vox_fbank_num_frames(int64_t num_samples, const vox_fbank_opts* o);
/* n_utt waveforms concatenated in d_wav (float sample values as Kaldi reads
 * int16 wavs); d_samp_off / d_frame_off: device int64[n_utt + 1] prefix offsets
 * of samples / frames (frames from vox_fbank_num_frames).  Writes
 * d_out[total_frames][num_mel_bins] float32.  Asynchronous on `stream`.
 * Replaces compute-fbank-feats (Kaldi feature-fbank.cc, not vendored). */
int vox_fbank_device(const float* d_wav, const int64_t* d_samp_off, const int64_t* d_frame_off,
                     int n_utt, int64_t total_frames, const vox_fbank_opts* o, float* d_out,
                     void* stream);
/* As vox_fbank_device, with d_utt_key: device uint64[n_utt] per-utterance
 * dither keys (e.g. a hash of the utterance id), so every utterance draws its
 * own noise -- as Kaldi's per-utterance RandomState does -- while the result
 * stays independent of batch composition.  d_utt_key == NULL is
 * vox_fbank_device (noise a function of seed, frame and sample only). */
int vox_fbank_device_keyed(const float* d_wav, const int64_t* d_samp_off,
                           const int64_t* d_frame_off, const uint64_t* d_utt_key, int n_utt,
                           int64_t total_frames, const vox_fbank_opts* o, float* d_out,
                           void* stream);
/* Sliding-window CMN of n_utt feature matrices [frames][f] concatenated in
 * d_in (frame offsets d_frame_off[n_utt + 1]); bit-identical to
 * vox_sliding_cmn per utterance.  Replaces `apply-cmvn-sliding` (tf_extract.py:63). */
int vox_sliding_cmn_device(const float* d_in, const int64_t* d_frame_off, int n_utt, int f,
                           int cmn_window, int center, float* d_out, void* stream);
/* Kaldi CompressedMatrix round trip of n_utt feature matrices [frames][f]
 * concatenated in d_in (`copy-feats --compress=true`, prepare_data.sh:69,
 * method kAutomaticMethod: "CM " kSpeechFeature for rows > 8, "CM2 "
 * kTwoByteAuto otherwise).  Writes each utterance's compressed payload (the
 * bytes after the "CM " / "CM2 " token, vox_cm_blob_bytes(rows, f) of them) at
 * d_blob + d_blob_off[u] (device int64[n_utt]) and, when d_out is non-NULL, the
 * decoded features as Kaldi's CopyToMat yields them (the matrix
 * apply-cmvn-sliding reads).  Asynchronous on `stream`.  n_utt <= 65535. */
int64_t vox_cm_blob_bytes(int rows, int cols);
int vox_cm_compress_device(const float* d_in, const int64_t* d_frame_off, int n_utt, int f,
                           uint8_t* d_blob, const int64_t* d_blob_off, float* d_out, void* stream);
/* The device side of the extraction reader (tf_extract.py:63: apply-cmvn-sliding
 * over the `copy-feats --compress` arks, prepare_data.sh:69), the GPU form of
 * vox_read_chunks(_ragged) for "CM " matrices: U payloads as
 * vox_read_cm_payloads reads them are decoded in Kaldi C++'s arithmetic
 * (bit-identical to vox_read_mat_kaldi), sliding-window CMN'd when
 * cmn_window > 0 (centered; bit-identical to vox_sliding_cmn), and n_items
 * chunks gathered into d_out [n_items][stride][f] (rows past a chunk's length
 * zero).  d_meta (device int64): blob_off[U+1] | frame_off[U+1] | rows[U] |
 * item_utt[n] | item_start[n] | item_len[n]; utterance u's payload at
 * d_blob + blob_off[u] holds rows[u] rows, of which the first need[u] =
 * frame_off[u+1] - frame_off[u] are decoded (total_rows = frame_off[U],
 * max_need = the largest need).  The CMN windows of a chunk's rows must lie in
 * the decoded rows: need = min(rows, max(end + cmn_window - cmn_window/2,
 * cmn_window)) for the utterance's last chunk end `end` (need = end without
 * CMN).  d_work: 2 * total_rows * f floats (total_rows * f without CMN).
 * Asynchronous on `stream`; U <= 65535. */
int vox_cm_chunks_device(const uint8_t* d_blob, const int64_t* d_meta, int n_utt,
                         int64_t total_rows, int max_need, int n_items, int stride, int f,
                         int cmn_window, float* d_work, float* d_out, void* stream);

const char* vox_last_error(void);

/* ---- layer-by-layer parity support (tests, not the extraction path) ------
 * The plan at (n, t) for the device buffers (d_x, d_out) is a sequence of
 * kernel launches; after launches [0, op_end) of tap i have run, `data` holds
 * layer i's output (NHWC [n,h,w,c], row stride `ld` elements, dtype VOX_BF16 /
 * VOX_FP32 = the model precision).  Layers are the oracle's boundaries
 * (oracle/models_ref.py `layers`): the stem / first TDNN layer, every
 * bottleneck / DPN block / TDNN layer; the remaining launches are pooling and
 * the head.  vox_debug_taps returns the tap count (fills up to max_taps) and
 * the number of launches of the whole plan in *n_ops;
 * vox_debug_run_ops runs launches [op_begin, op_end) eagerly and synchronises;
 * vox_debug_read copies device bytes to the host. */
typedef struct vox_tap {
  int op_end;
  int n, h, w, c, ld;
  int dtype;
  const void* data;
} vox_tap;
int vox_debug_taps(vox_model* m, const float* d_x, int n, int t, int f, float* d_out,
                   vox_tap* taps, int max_taps, int* n_ops);
int vox_debug_run_ops(vox_model* m, int op_begin, int op_end, void* stream);
int vox_debug_read(void* dst, const void* d_src, size_t bytes);
/* sizeof of an internal kernel parameter struct (0 = BneckParams, 1 = GconvParams),
 * for tests that launch a kernel through a ctypes mirror of it; -1 otherwise. */
int64_t vox_debug_struct_size(int which);

/* ---- host-side Kaldi I/O (no Kaldi binaries needed) --------------------- */
int vox_sliding_cmn(const float* in, int t, int f, int cmn_window, int center,
                    float* out);
/* Binary Kaldi matrix ("\0B" + FM/DM/CM) at byte `offset` of `path`. */
int vox_mat_shape(const char* path, int64_t offset, int* rows, int* cols);
int vox_read_mat(const char* path, int64_t offset, float* out, int rows, int cols);
/* Same, from memory: `buf` starts at "\0B". */
int vox_parse_mat(const uint8_t* buf, size_t nbytes, float* out, int rows, int cols,
                  size_t* consumed);
int vox_parse_mat_shape(const uint8_t* buf, size_t nbytes, int* rows, int* cols);
/* The same two readers with CM payloads decoded in Kaldi C++'s arithmetic
 * (CompressedMatrix::Uint16ToFloat / CharToFloat) instead of kaldi_io's: what
 * the reference's `apply-cmvn-sliding ark:...` pipe (tf_extract.py:63) decodes
 * from the `copy-feats --compress` arks (prepare_data.sh:69).  FM/DM: identical. */
int vox_read_mat_kaldi(const char* path, int64_t offset, float* out, int rows, int cols);
int vox_parse_mat_kaldi(const uint8_t* buf, size_t nbytes, float* out, int rows, int cols,
                        size_t* consumed);
/* Batched reader of the extraction path (the tf_extract.py get_batch process
 * and its apply-cmvn-sliding rspec pipe, :63,:85-90) on `threads` host threads.
 * vox_mat_shapes: rows/cols of n matrices at paths[i]:offsets[i], headers only.
 * vox_read_chunks: one batch of n equal-length chunks -- item i is rows
 * [r0[i], r0[i] + T[i]) and columns [c0[i], c0[i] + f) of the matrix at
 * paths[i]:offsets[i] (an scp rxfile with its optional [range]; CM decoded in
 * Kaldi C++'s arithmetic), sliding CMN over those T[i] rows when cmn_window > 0
 * (window cmn_window, centered; bit-identical to vox_sliding_cmn of the whole
 * utterance), then frames [start[i], start[i] + len) into out + i*len*f. */
int vox_mat_shapes(const char* const* paths, const int64_t* offsets, int n, int* rows, int* cols,
                   int threads);
int vox_read_chunks(const char* const* paths, const int64_t* offsets, const int* r0, const int* T,
                    const int* c0, const int* start, int n, int f, int len, int cmn_window,
                    float* out, int threads);
/* The same for a ragged batch (vox_embed_lens): item i has lens[i] frames
 * (1 <= lens[i] <= stride) and goes to out + i*stride*f; its rows from lens[i]
 * to stride are left untouched (padding). */
int vox_read_chunks_ragged(const char* const* paths, const int64_t* offsets, const int* r0,
                           const int* T, const int* c0, const int* start, const int* lens, int n,
                           int f, int stride, int cmn_window, float* out, int threads);
/* Matrix kinds at paths[i]:offsets[i] (headers only): 0 "FM", 1 "DM", 2 "CM",
 * 3 "CM2". */
int vox_mat_kinds(const char* const* paths, const int64_t* offsets, int n, int* kinds, int threads);
/* The raw "CM " payloads (the bytes after the token) of n matrices into buf:
 * payload i at buf + blob_off[i], blob_off[i+1] - blob_off[i] = 16 + 8 cols +
 * rows cols bytes (rows > 8) -- the input of vox_cm_chunks_device.  VOX_EINVAL
 * when a matrix is not "CM " with those dimensions. */
int vox_read_cm_payloads(const char* const* paths, const int64_t* offsets, int n,
                         const int64_t* blob_off, int cols, uint8_t* buf, int threads);
/* Serialise "key \0BFV \4<u32 dim><dim f32>" into buf; returns bytes written
 * (or needed, if cap is too small) and the offset of "\0B" via *data_offset. */
int64_t vox_format_vec_flt(const char* key, const float* v, int dim, uint8_t* buf,
                           size_t cap, int64_t* data_offset);

#ifdef __cplusplus
}
#endif
#endif /* VOXEMB_H */
