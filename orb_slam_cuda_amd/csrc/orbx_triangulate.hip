// orbx_triangulate.hip — ORBmatcher::SearchForTriangulation on the GPU
// (src/ORBmatcher.cc:657-823, CheckDistEpipolarLine :140-157; called by
// LocalMapping::CreateNewMapPoints for the new keyframe against each of its
// best covisible keyframes).
//
// For every keypoint idx1 of pKF1 without a MapPoint (stereo only when
// bOnlyStereo) in a vocabulary node that pKF2's FeatureVector also holds,
// the candidates are pKF2's keypoints of that node without a MapPoint; a
// candidate is taken when its Hamming distance is <= TH_LOW and <= the best
// so far (so the LAST candidate at the minimal distance wins), it is not
// near the epipole (both monocular) and it lies within 3.84 sigma^2 of the
// epipolar line of F12. The reference declares vbMatched2 (:680) but never
// sets it, so the idx1 searches are independent: one lane per idx1. The
// rotation-consistency check (three largest bins) then clears matches.
//
// One 256-thread workgroup per keyframe pair; a batch of pairs (the new
// keyframe against its neighbours) is one launch.
#include "orbx_projgrid.cuh"

namespace orbx {

constexpr int kTriThreads = 256;
constexpr int kTriHisto = 30;  // HISTO_LENGTH
constexpr int kTriThLow = 50;  // TH_LOW

__global__ __launch_bounds__(kTriThreads) void search_tri_kernel(TriParams P, TriSide A, TriSide B,
                                                                 const orbm_tri_pair* __restrict__ pairs,
                                                                 int* __restrict__ matches12,
                                                                 int* __restrict__ nmatches) {
  __shared__ int s_hist[kTriHisto], s_ind[3], s_cnt, s_rej;
  const int p = blockIdx.x, tid = threadIdx.x, lane = tid & 63;
  const size_t ka = (size_t)p * A.kp_pitch, kb = (size_t)p * B.kp_pitch;
  const size_t na = (size_t)p * A.node_pitch, nb = (size_t)p * B.node_pitch;
  const orbx_kp* kp1 = A.kps + ka;
  const uint8_t* d1 = A.desc + ka * 32;
  const float* ur1 = A.uright + ka;
  const uint8_t* mp1 = A.has_mp + ka;
  const uint32_t* nodes1 = A.nodes + na;
  const int* off1 = A.off + na + (A.node_pitch ? p : 0);  // off arrays hold node_pitch + 1 entries per pair
  const int* idx1s = A.idx + ka;
  const int nn1 = A.nn[A.kp_pitch ? p : 0], n1 = A.n[A.kp_pitch ? p : 0];
  const orbx_kp* kp2 = B.kps + kb;
  const uint8_t* d2 = B.desc + kb * 32;
  const float* ur2 = B.uright + kb;
  const uint8_t* mp2 = B.has_mp + kb;
  const uint32_t* nodes2 = B.nodes + nb;
  const int* off2 = B.off + nb + (B.node_pitch ? p : 0);
  const int* idx2s = B.idx + kb;
  const int nn2 = B.nn[p];
  const orbm_tri_pair T = pairs[p];
  int* M = matches12 + (size_t)p * P.out_pitch;

  for (int i = tid; i < n1; i += kTriThreads) M[i] = -1;
  if (tid < kTriHisto) s_hist[tid] = 0;
  if (tid == 0) {
    s_cnt = 0;
    s_rej = 0;
  }
  __syncthreads();
  const int npos = off1[nn1];
  const float factor = 1.0f / kTriHisto;
  int cnt = 0;
  for (int q = tid; q < npos; q += kTriThreads) {
    // node of CSR position q: the last k with off1[k] <= q
    int lo = 0, hi = nn1 - 1;
    while (lo < hi) {
      const int mid = (lo + hi + 1) >> 1;
      if (off1[mid] <= q) lo = mid;
      else hi = mid - 1;
    }
    const uint32_t id = nodes1[lo];
    int a = 0, b = nn2;  // lower_bound in pKF2's nodes
    while (a < b) {
      const int mid = (a + b) >> 1;
      if (nodes2[mid] < id) a = mid + 1;
      else b = mid;
    }
    if (a >= nn2 || nodes2[a] != id) continue;
    const int i1 = idx1s[q];
    if (mp1[i1]) continue;  // pKF1->GetMapPoint(idx1)
    const bool st1 = ur1[i1] >= 0.0f;
    if (P.only_stereo && !st1) continue;
    const orbx_kp k1 = kp1[i1];
    const uint4* dd1 = (const uint4*)(d1 + (size_t)i1 * 32);
    const uint4 m0 = dd1[0], m1 = dd1[1];
    // epipolar line of kp1 in image 2: l = x1' F12 (CheckDistEpipolarLine :143-145)
    const float la = __fadd_rn(__fadd_rn(__fmul_rn(k1.x, T.F12[0]), __fmul_rn(k1.y, T.F12[3])), T.F12[6]);
    const float lb = __fadd_rn(__fadd_rn(__fmul_rn(k1.x, T.F12[1]), __fmul_rn(k1.y, T.F12[4])), T.F12[7]);
    const float lc = __fadd_rn(__fadd_rn(__fmul_rn(k1.x, T.F12[2]), __fmul_rn(k1.y, T.F12[5])), T.F12[8]);
    const float den = __fadd_rn(__fmul_rn(la, la), __fmul_rn(lb, lb));
    int bestDist = kTriThLow, bestIdx2 = -1;
    for (int r = off2[a]; r < off2[a + 1]; ++r) {
      const int i2 = idx2s[r];
      if (mp2[i2]) continue;  // vbMatched2[idx2] is never set
      const bool st2 = ur2[i2] >= 0.0f;
      if (P.only_stereo && !st2) continue;
      const uint4* dd2 = (const uint4*)(d2 + (size_t)i2 * 32);
      const int dist = hamming256(dd2[0], dd2[1], m0, m1);
      if (dist > kTriThLow || dist > bestDist) continue;
      const orbx_kp k2 = kp2[i2];
      const int o2 = min(max(k2.octave, 0), kMaxLevels - 1);
      if (!st1 && !st2) {
        const float dx = __fsub_rn(T.ex, k2.x), dy = __fsub_rn(T.ey, k2.y);
        if (__fadd_rn(__fmul_rn(dx, dx), __fmul_rn(dy, dy)) < __fmul_rn(100.0f, P.scale2[o2])) continue;
      }
      if (den == 0.0f) continue;
      const float num = __fadd_rn(__fadd_rn(__fmul_rn(la, k2.x), __fmul_rn(lb, k2.y)), lc);
      const float dsqr = __fdiv_rn(__fmul_rn(num, num), den);
      if ((double)dsqr < 3.84 * (double)P.sigma2[o2]) {
        bestIdx2 = i2;
        bestDist = dist;
      }
    }
    if (bestIdx2 >= 0) {
      M[i1] = bestIdx2;
      ++cnt;
      if (P.check_ori) {
        float rot = __fsub_rn(k1.angle, kp2[bestIdx2].angle);
        if (rot < 0.0f) rot = __fadd_rn(rot, 360.0f);
        int bin = (int)roundf(__fmul_rn(rot, factor));
        if (bin == kTriHisto) bin = 0;
        atomicAdd(&s_hist[bin], 1);
      }
    }
  }
  cnt = wave_sum_dpp(cnt);
  if (lane == 0 && cnt) atomicAdd(&s_cnt, cnt);
  __syncthreads();
  if (P.check_ori) {
    if (tid == 0) {  // ComputeThreeMaxima (:1601-1642)
      int max1 = 0, max2 = 0, max3 = 0, ind1 = -1, ind2 = -1, ind3 = -1;
      for (int i = 0; i < kTriHisto; i++) {
        const int s = s_hist[i];
        if (s > max1) {
          max3 = max2; max2 = max1; max1 = s;
          ind3 = ind2; ind2 = ind1; ind1 = i;
        } else if (s > max2) {
          max3 = max2; max2 = s;
          ind3 = ind2; ind2 = i;
        } else if (s > max3) {
          max3 = s;
          ind3 = i;
        }
      }
      if (max2 < __fmul_rn(0.1f, (float)max1)) {
        ind2 = -1;
        ind3 = -1;
      } else if (max3 < __fmul_rn(0.1f, (float)max1)) {
        ind3 = -1;
      }
      s_ind[0] = ind1;
      s_ind[1] = ind2;
      s_ind[2] = ind3;
    }
    __syncthreads();
    int rej = 0;
    for (int i = tid; i < n1; i += kTriThreads) {
      const int j = M[i];
      if (j < 0) continue;
      float rot = __fsub_rn(kp1[i].angle, kp2[j].angle);
      if (rot < 0.0f) rot = __fadd_rn(rot, 360.0f);
      int bin = (int)roundf(__fmul_rn(rot, factor));
      if (bin == kTriHisto) bin = 0;
      if (bin == s_ind[0] || bin == s_ind[1] || bin == s_ind[2]) continue;
      M[i] = -1;
      ++rej;
    }
    rej = wave_sum_dpp(rej);
    if (lane == 0 && rej) atomicAdd(&s_rej, rej);
    __syncthreads();
  }
  if (tid == 0) nmatches[p] = s_cnt - s_rej;
}

int launch_search_tri(const TriParams& P, const TriSide& A, const TriSide& B, const orbm_tri_pair* pairs, int npairs,
                      int* matches12, int* nmatches, void* stream) {
  hipLaunchKernelGGL(search_tri_kernel, dim3(npairs), dim3(kTriThreads), 0, (hipStream_t)stream, P, A, B, pairs,
                     matches12, nmatches);
  return hipGetLastError() == hipSuccess ? ORBX_OK : ORBX_EDEVICE;
}

}  // namespace orbx
