// orbx_extract.hip — the batched ORBextractor::operator() pipeline for gfx950.
//
// For a batch of B frames, all on one stream, no host round trip:
//   launch_pyramid       (1, or L-1 launches) ComputePyramid        orbx_pyramid.hip
//   launch_blur          (1)  GaussianBlur 7x7 s=2                  orbx_blur.hip
//   launch_fast          (1)  per-cell FAST + NMS                   orbx_fast.hip
//   launch_quadtree      (1)  DistributeOctTree                     orbx_quadtree.hip
//   launch_orient_brief  (1)  IC_Angle + rBRIEF + scale/assemble    orbx_brief.hip
// Optional events (caller-owned or the handle's ORBX_TIMING ones) bracket
// every stage on the launch stream (ev[i], ev[i+1] around stage i).
#include <cstdlib>
#include <cstring>

#include "orbx_device.cuh"

namespace orbx {

// Stage launch order: p pyramid, b blur, f FAST, q quadtree, o orient+BRIEF;
// the pyramid first, FAST before the quadtree, both the blur and the
// quadtree before orient+BRIEF, orient+BRIEF last. The stages' results do not
// depend on it; how a launch interleaves with other streams' work does. Default
// "pfqbo": the quadtree right behind FAST, the blur (read only by
// orient+BRIEF) after it (pipelined C3 172.5 -> 174.4 k frames/s, KITTI14
// 151.8 -> 159.0 k against "pbfqo"). ORBX_EXTRACT_ORDER
// overrides the default, orbx_set_stage_order a handle's. Stage event i + 1
// closes the i-th stage launched.
bool valid_stage_order(const char* e) {
  return e && strlen(e) == 5 && e[0] == 'p' && e[4] == 'o' && strchr(e, 'b') && strchr(e, 'f') && strchr(e, 'q') &&
         strchr(e, 'q') > strchr(e, 'f');
}
const char* extract_stage_order() {
  static const char* order = [] {
    const char* e = getenv("ORBX_EXTRACT_ORDER");
    return valid_stage_order(e) ? e : "pfqbo";
  }();
  return order;
}

int launch_extract(const ExtractParams& P, const ExtractBuffers& X, const uint8_t* d_frames, int batch,
                   size_t frame_pitch, size_t row_stride, orbx_kp* d_kps, uint8_t* d_desc, int* d_counts,
                   void* stream_, void** ev, void* pyr_event, int* status_dst, const char* stage_order) {
  hipStream_t stream = (hipStream_t)stream_;
  ExtractParams Q = P;
  Q.B = batch;
  Q.status_src = status_dst ? X.err : nullptr;
  Q.status_dst = status_dst;
  LevelPtrs lp;
  lp.base[0] = d_frames;
  lp.fstride[0] = (long long)frame_pitch;
  lp.pitch[0] = (int)row_stride;
  lp.aligned16[0] = ((((uintptr_t)d_frames) | frame_pitch | row_stride) & 15) == 0;
  for (int l = 1; l < P.L; ++l) {
    lp.base[l] = X.pyr + P.lv[l].off;
    lp.fstride[l] = P.lv[l].plane;
    lp.pitch[l] = P.lv[l].pitch;
    lp.aligned16[l] = 1;  // 64-byte pitches in a hipMalloc'ed buffer
  }
  auto rec = [&](int i) {
    if (ev) (void)hipEventRecord((hipEvent_t)ev[i], stream);
  };
  const char* order = stage_order ? stage_order : extract_stage_order();
  int rc;
  rec(0);
  for (int i = 0; i < 5; ++i) {
    switch (order[i]) {
      case 'p': rc = launch_pyramid(Q, lp, X.rtab, batch, stream); break;
      case 'b': rc = launch_blur(Q, lp, X.rtab, X.blur, batch, stream); break;
      case 'f': rc = launch_fast(Q, lp, X.cells, X.slots, X.cell_counts, batch, stream); break;
      case 'q': rc = launch_quadtree(Q, X, batch, stream); break;
      default: rc = launch_orient_brief(Q, lp, X, d_kps, d_desc, d_counts, batch, stream); break;
    }
    if (rc) return rc;
    if (order[i] == 'p' && pyr_event && hipEventRecord((hipEvent_t)pyr_event, stream) != hipSuccess)
      return ORBX_EDEVICE;
    rec(i + 1);
  }
  return ORBX_OK;
}

}  // namespace orbx
