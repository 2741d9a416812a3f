/* eray_hip_debug.h — test-only diagnostics exported by liberay_hip.so.
 *
 * Not part of the drop-in boundary (include/eray_hip.h): none of these replaces a reference
 * interface, and none is called by the library's own paths.  They exist for tests/ and scripts/:
 * each SYNCHRONISES the context's stream and copies device state to the host, so no production
 * caller should use them.  Status codes as in eray_hip.h.
 */
#ifndef ERAY_HIP_DEBUG_H
#define ERAY_HIP_DEBUG_H

#include "eray_hip.h"

#ifdef __cplusplus
extern "C" {
#endif

/* The screen bins of object `index` as built by the last setup: out[0] bins, out[1] entries,
 * out[2] (face, pixel) pairs, out[3] most entries in one bin, out[4] non-empty bins, out[5] most
 * pairs in one bin, out[6..9] the object's pixel rectangle, out[10] the fullest bin, out[11] /
 * out[12] bins of more than 64 / 192 entries, out[13] the units the pair pass walked (the faces'
 * bin-rectangle rows, or their (face, bin) pairs) (14 words). */
int eray_debug_bin_stats(eray_ctx* ctx, uint32_t index, uint64_t* out);
/* The entries of bin `bin` of object `index` (faces relative to the object, pixel masks), at most
 * `cap`; *n = the bin's entry count. */
int eray_debug_bin_dump(eray_ctx* ctx, uint32_t index, uint32_t bin, uint32_t* tri, uint64_t* mask, uint32_t cap,
                        uint32_t* n);
/* The same entries with their pad words (`pad` may be null): in a bin of 65..1024 entries (sorted by
 * face), entries 64 c and 64 c + 1 hold the low / high half of the union of the masks of chunks
 * c + 1 .. (render.hip first_hit_binned_wave's early end); every other pad is 0. */
int eray_debug_bin_entries(eray_ctx* ctx, uint32_t index, uint32_t bin, uint32_t* tri, uint64_t* mask, uint32_t* pad,
                           uint32_t cap, uint32_t* n);
/* The frame setups' pair pass over every (face, bin) pair of the faces' bin rectangles
 * (rect_pairs != 0) instead of the rectangles' rows; the next setup rebuilds the bins. */
int eray_debug_set_bin_form(eray_ctx* ctx, int rect_pairs);
/* Sets the bins' entry capacity (reallocated at the next setup; overflow and growth tests). */
int eray_debug_set_bin_capacity(eray_ctx* ctx, uint64_t entries);
uint64_t eray_debug_bin_capacity(const eray_ctx* ctx);
/* The last setup's device state (192 B) and object `index`'s pixel rectangle. */
int eray_debug_setup_state(eray_ctx* ctx, uint32_t index, void* state_out, int32_t* rect_out);
/* The multi-GPU gathers' rank-0 steps for N ranks simulated on one GPU (staging: the N ranks'
 * padded local PPM blocks): the band reorder, the coded transport's decode, the scene-camera
 * gather's pack + assemble. */
int eray_debug_unband(eray_ctx* ctx, const uint8_t* staging, uint8_t* frame, uint32_t height, uint32_t width,
                      uint32_t band_rows, uint32_t nranks);
int eray_debug_coded_unband(eray_ctx* ctx, const uint8_t* staging, uint8_t* frame, uint32_t height, uint32_t width,
                            uint32_t band_rows, uint32_t nranks);
int eray_debug_scene_gather(eray_ctx* ctx, const uint8_t* staging, uint8_t* frame, uint32_t height, uint32_t width,
                            uint32_t band_rows, uint32_t nranks);
/* A batch of nframes frames (frame k of rank q at staging block k * nranks + q) with every rank's
 * transfer schedule played as device copies; rotate: ERAY_GATHER_ROTATE_ROOT's roots.  Root r's
 * frames land at frames + (frames of roots below r + j) * height * width * 3. */
int eray_debug_scene_gather_batch(eray_ctx* ctx, const uint8_t* staging, uint8_t* frames, uint32_t nframes,
                                  uint32_t height, uint32_t width, uint32_t band_rows, uint32_t nranks, uint32_t rotate);
/* Host only: rank `rank`'s part of a batch's scene-camera gather when rank q packs rank_bytes[q]
 * bytes per frame.  out (u64, cap >= 5 + nframes + 12 nranks): buffer bytes, frames it assembles,
 * transfer count T; per frame its pack's offset in the buffer; per rank q the receive offset of
 * q's packs; per transfer peer, 1 send / 0 receive, offset, bytes (a transfer ends with its
 * sender's 16-byte header); the number of headers the rank writes and their offsets (T + 1
 * slots); per rank q the offset of q's header in the rank's receive area (~0: unused). */
int eray_debug_gather_schedule(const uint32_t* rank_bytes, uint32_t nranks, uint32_t rank, uint32_t nframes,
                               uint32_t rotate, uint64_t* out, uint32_t cap);
/* Host only: the headers rank `rank` writes into (a host copy of) its transfer buffer — its own
 * verdict `status` and its frames' source (kind, key) — and a root's verdict on a received
 * buffer (every header it uses ERAY_OK and the plan's source; else ERAY_E_INVALID_ARGUMENT and the
 * root writes none of the batch's frames). */
int eray_debug_gather_write_headers(const uint32_t* rank_bytes, uint32_t nranks, uint32_t rank, uint32_t nframes,
                                    uint32_t rotate, int32_t status, uint32_t kind, uint64_t key, uint8_t* buf);
int eray_debug_gather_check(const uint32_t* rank_bytes, uint32_t nranks, uint32_t rank, uint32_t nframes,
                            uint32_t rotate, uint32_t kind, uint64_t key, const uint8_t* buf);
/* Host only: a new gather plan's verdict on rank `rank` from every rank's exchange record
 * (status, kind, key low, key high; 4 words each) — all ranks accept or all fail together. */
int eray_debug_plan_verdict(const int32_t* records, uint32_t nranks, uint32_t rank);
/* The entry count of every screen bin of object `index` as built for the last setup (row-major
 * over the camera's bin rows, at most `cap`); *nbins receives the bin count.  Synchronises. */
int eray_debug_bin_counts(eray_ctx* ctx, uint32_t index, uint32_t* counts, uint32_t cap, uint32_t* nbins);
/* Host only: eray_gather_frames' re-plan decision from its only inputs — whether the cached plan
 * fits the call's shared arguments, the plan's source (kind, key) and the context's latest
 * scene-camera / camera-path render's — 1: a new plan is exchanged, 0: the cached one is used. */
int eray_debug_gather_replan(uint32_t cached, uint32_t plan_kind, uint64_t plan_key, uint32_t cur_kind,
                             uint64_t cur_key);
/* Host only (no context, no GPU): rank `rank`'s share of the scene-camera gather of `nranks` ranks
 * for objects whose pixel rectangles are `rects` (n x (x0, x1, y0, y1), camera rows) — its rows, its
 * rectangles in local rows / 16-pixel column groups, each one's offset in its per-frame pack.  out:
 * 4 + 8 x 8 words (rows, nrect, bytes per frame, packed rows, then per rectangle l0, l1, c0, c1,
 * offset, row bytes, first packed row, 0). */
int eray_debug_gather_layout(const int32_t* rects, uint32_t n, uint32_t height, uint32_t width, uint32_t band_rows,
                             uint32_t nranks, uint32_t rank, uint32_t* out);

#ifdef __cplusplus
}
#endif
#endif /* ERAY_HIP_DEBUG_H */
