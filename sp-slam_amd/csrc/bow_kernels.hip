// Bag of words on gfx950:
//   Frame::ComputeBoW (src/Frame.cc:495-502) = DBoW2 TemplatedVocabulary::transform
//     (features, BowVector, FeatureVector, levelsup = 4) (TemplatedVocabulary.h:1127-1194,
//     per feature :1217-1259; BowVector.cpp addWeight / addIfNotExist / normalize;
//     FeatureVector.cpp addFeature; FORB::distance);
//   ORBmatcher::SearchByBoW(KeyFrame*, Frame&, vector<MapPoint*>&) (src/ORBmatcher.cc:159-288).
// Semantics: oracle/bow_oracle.cpp.
//
//   bow_words_kernel    thread per feature: descend the vocabulary tree (first minimum
//                       of the 256-bit Hamming distance over each node's children, in
//                       the loaded order) -> word id, weight, node at level L - levelsup.
//                       The top of the tree is read by every feature and stays in L2.
//   bow_vectors_kernel  workgroup per frame: bitonic sort of (word, feature) keys in LDS,
//                       one thread per run sums its weights in feature order (the
//                       std::map += order), the L1 / L2 norm in word order by one thread
//                       (the reference's map walk; <= cap dependent fp64 adds), then the
//                       (node, feature) sort gives the FeatureVector as CSR.
//   bow_search_kernel   workgroup per (keyframe, frame) pair: shared FeatureVector nodes
//                       are independent (a frame feature sits in one node), so each wave
//                       takes whole nodes; inside a node the keyframe features run in
//                       order (a match takes the frame feature for the later ones) and the
//                       64 lanes split the node's frame features, reducing (best, first
//                       index, second best) exactly as the sequential `<` scan; rotation
//                       histogram + ComputeThreeMaxima at the end.
// Integer / index work and fp64 sums in the reference's order: bit-exact.
#include <hip/hip_runtime.h>

#include "bow_launch.h"

namespace spslam {
namespace bow {

constexpr int kThreads = 256;
constexpr int kHisto = 30, kThLow = 50;

__device__ __forceinline__ int hamming(const uint4& a0, const uint4& a1, const uint4& b0, const uint4& b1) {
    return __popc(a0.x ^ b0.x) + __popc(a0.y ^ b0.y) + __popc(a0.z ^ b0.z) + __popc(a0.w ^ b0.w) +
           __popc(a1.x ^ b1.x) + __popc(a1.y ^ b1.y) + __popc(a1.z ^ b1.z) + __popc(a1.w ^ b1.w);
}

__global__ __launch_bounds__(kThreads) void bow_words_kernel(VocabDev V, const uint8_t* __restrict__ desc,
                                                             const int* __restrict__ counts, int cap, int n_frames,
                                                             int nid_level, uint32_t* __restrict__ s_word,
                                                             double* __restrict__ s_weight,
                                                             uint32_t* __restrict__ s_node) {
    const long long g = (long long)blockIdx.x * kThreads + threadIdx.x;
    if (g >= (long long)n_frames * cap) return;
    const int f = (int)(g / cap), i = (int)(g - (long long)f * cap);
    if (i >= min(counts[f], cap)) return;
    const uint4* p = reinterpret_cast<const uint4*>(desc + g * 32);
    const uint4 a0 = p[0], a1 = p[1];
    int node = 0, level = 0;
    uint32_t nid = 0;
    bool set = nid_level <= 0;
    int cc = V.child_count[0];
    do {
        ++level;
        const int cb = V.child_begin[node];
        int best = V.child_ids[cb];
        int bd = hamming(a0, a1, V.desc[2 * best], V.desc[2 * best + 1]);
        for (int c = 1; c < cc; c++) {
            const int id = V.child_ids[cb + c];
            const int d = hamming(a0, a1, V.desc[2 * id], V.desc[2 * id + 1]);
            if (d < bd) {
                bd = d;
                best = id;
            }
        }
        node = best;
        if (level == nid_level) {
            nid = (uint32_t)node;
            set = true;
        }
        cc = V.child_count[node];
    } while (cc > 0);
    if (!set) nid = (uint32_t)node;  // indeterminate in the reference (oracle header)
    s_word[g] = V.word_id[node];
    s_weight[g] = V.weight[node];
    s_node[g] = nid;
}

// ascending bitonic sort of P (power of two) 64-bit keys in LDS
__device__ void bitonic_sort(unsigned long long* key, int P) {
    for (int k = 2; k <= P; k <<= 1) {
        for (int j = k >> 1; j > 0; j >>= 1) {
            for (int t = threadIdx.x; t < P; t += kThreads) {
                const int q = t ^ j;
                if (q > t) {
                    const unsigned long long x = key[t], y = key[q];
                    const bool up = (t & k) == 0;
                    if ((x > y) == up) {
                        key[t] = y;
                        key[q] = x;
                    }
                }
            }
            __syncthreads();
        }
    }
}

// exclusive prefix over threads of `v`; returns this thread's offset, *total the sum
__device__ int block_exclusive_scan(int v, int* tmp, int* total) {
    const int t = threadIdx.x;
    tmp[t] = v;
    __syncthreads();
    for (int o = 1; o < kThreads; o <<= 1) {
        const int add = t >= o ? tmp[t - o] : 0;
        __syncthreads();
        tmp[t] += add;
        __syncthreads();
    }
    const int incl = tmp[t];
    *total = tmp[kThreads - 1];
    __syncthreads();
    return incl - v;
}

__global__ __launch_bounds__(kThreads) void bow_vectors_kernel(int cap, int P, int tf, int must, int l2,
                                                               const int* __restrict__ counts,
                                                               const uint32_t* __restrict__ s_word,
                                                               const double* __restrict__ s_weight,
                                                               const uint32_t* __restrict__ s_node, BowOut out) {
    extern __shared__ unsigned long long lds[];
    unsigned long long* key = lds;                          // [P]
    double* vals = reinterpret_cast<double*>(lds + P);      // [P]
    __shared__ int scan_tmp[kThreads];
    __shared__ double norm_s;
    const int f = blockIdx.x, t = threadIdx.x;
    const size_t fo = (size_t)f * cap;
    const int n = min(counts[f], cap);
    const int per = P / kThreads > 0 ? P / kThreads : 1;   // contiguous elements per thread
    const int lo = min(t * per, P), hi = min(lo + per, P);
    // keys at positions >= n are ~0 (the maximum), so sorting the first power of two >= n gives the full sort's
    // array: a frame with few features (none, when the caller masks it) does not pay for cap
    int Pn = n > 0 ? 1 : 0;
    while (Pn < n) Pn <<= 1;
    Pn = min(Pn, P);

    // ---- BowVector: (word, feature) keys of the features that are not stop words
    int valid = 0;
    for (int q = t; q < P; q += kThreads) {
        const bool ok = q < n && s_weight[fo + q] > 0.0;
        key[q] = ok ? ((unsigned long long)s_word[fo + q] << 32) | (unsigned)q : ~0ull;
        valid += ok;
    }
    int m;
    block_exclusive_scan(valid, scan_tmp, &m);
    bitonic_sort(key, Pn);
    int heads = 0;
    for (int q = lo; q < hi; q++)
        heads += q < m && (q == 0 || (key[q] >> 32) != (key[q - 1] >> 32));
    int nb;
    int u = block_exclusive_scan(heads, scan_tmp, &nb);
    for (int q = lo; q < hi; q++) {
        if (!(q < m && (q == 0 || (key[q] >> 32) != (key[q - 1] >> 32)))) continue;
        const unsigned w = (unsigned)(key[q] >> 32);
        double v = s_weight[fo + (unsigned)key[q]];
        if (tf)  // addWeight: += in feature order; addIfNotExist keeps the first
            for (int r = q + 1; r < m && (unsigned)(key[r] >> 32) == w; r++) v += s_weight[fo + (unsigned)key[r]];
        out.bow_words[fo + u] = w;
        vals[u++] = v;
    }
    __syncthreads();
    if (t == 0) {
        double norm = 0.0;
        if (must) {  // BowVector::normalize: the std::map walk in word order
            if (!l2) {
                for (int q = 0; q < nb; q++) norm += fabs(vals[q]);
            } else {
                for (int q = 0; q < nb; q++) norm += vals[q] * vals[q];
                norm = sqrt(norm);
            }
        }
        norm_s = norm;
        out.n_bow[f] = nb;
    }
    __syncthreads();
    const double norm = norm_s, nd = (double)nb;
    for (int q = t; q < nb; q += kThreads) {
        double v = vals[q];
        if (tf && !must) v /= nd;
        if (must && norm > 0.0) v /= norm;
        out.bow_values[fo + q] = v;
    }
    __syncthreads();

    // ---- FeatureVector: (node, feature) keys of the same features
    for (int q = t; q < P; q += kThreads) {
        const bool ok = q < n && s_weight[fo + q] > 0.0;
        key[q] = ok ? ((unsigned long long)s_node[fo + q] << 32) | (unsigned)q : ~0ull;
    }
    __syncthreads();
    bitonic_sort(key, Pn);
    heads = 0;
    for (int q = lo; q < hi; q++)
        heads += q < m && (q == 0 || (key[q] >> 32) != (key[q - 1] >> 32));
    int nf;
    u = block_exclusive_scan(heads, scan_tmp, &nf);
    int32_t* fv_start = out.fv_start + (size_t)f * (cap + 1);
    for (int q = lo; q < hi; q++) {
        if (q >= m) break;
        out.fv_features[fo + q] = (int32_t)(unsigned)key[q];
        if (q == 0 || (key[q] >> 32) != (key[q - 1] >> 32)) {
            out.fv_nodes[fo + u] = (uint32_t)(key[q] >> 32);
            fv_start[u++] = q;
        }
    }
    if (t == 0) {
        fv_start[nf] = m;
        out.n_fv[f] = nf;
    }
}

// ComputeThreeMaxima (src/ORBmatcher.cc:1601-1642)
__device__ void three_maxima(const int* h, int* i1, int* i2, int* i3) {
    int max1 = 0, max2 = 0, max3 = 0, ind1 = -1, ind2 = -1, ind3 = -1;
    for (int i = 0; i < kHisto; i++) {
        const int s = h[i];
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
    if (max2 < __fmul_rn(0.1f, (float)max1)) { ind2 = -1; ind3 = -1; }
    else if (max3 < __fmul_rn(0.1f, (float)max1)) ind3 = -1;
    *i1 = ind1; *i2 = ind2; *i3 = ind3;
}

// (best distance, its first position, second best) of a strided scan, merged across lanes
struct Best {
    int b1, i1, b2;
};

__device__ __forceinline__ Best merge(const Best& a, const Best& b) {
    Best r;
    if (a.b1 < b.b1 || (a.b1 == b.b1 && a.i1 < b.i1)) {
        r.b1 = a.b1; r.i1 = a.i1; r.b2 = min(a.b2, b.b1);
    } else {
        r.b1 = b.b1; r.i1 = b.i1; r.b2 = min(b.b2, a.b1);
    }
    return r;
}

__global__ __launch_bounds__(kThreads) void bow_search_kernel(const int2* __restrict__ pairs, BowSide K, BowSide F,
                                                              float nn_ratio, int check_ori,
                                                              int32_t* __restrict__ match_out,
                                                              int* __restrict__ nmatches_out) {
    extern __shared__ int smem[];
    int32_t* match = smem;                                          // [F.cap]
    int2* shared_nodes = reinterpret_cast<int2*>(smem + F.cap);     // [K.cap]
    signed char* bin = reinterpret_cast<signed char*>(shared_nodes + K.cap);  // [F.cap]
    __shared__ int hist[kHisto];
    __shared__ int n_shared, n_total, n_removed;
    __shared__ int ind[3];
    const int p = blockIdx.x, t = threadIdx.x, lane = t & 63, wave = t >> 6;
    const int kf = pairs[p].x, fr = pairs[p].y;
    const int nF = min(F.counts[fr], F.cap);
    for (int i = t; i < F.cap; i += kThreads) {
        match[i] = -1;
        bin[i] = -1;
    }
    if (t < kHisto) hist[t] = 0;
    if (t == 0) { n_shared = 0; n_total = 0; n_removed = 0; }
    __syncthreads();
    // nodes present in both FeatureVectors (processing order is free: the frame features of different
    // nodes are disjoint, so no node's outcome depends on another's)
    const uint32_t* kn = K.fv_nodes + (size_t)kf * K.cap;
    const uint32_t* fn = F.fv_nodes + (size_t)fr * F.cap;
    const int nk = K.n_fv[kf], nfv = F.n_fv[fr];
    for (int a = t; a < nk; a += kThreads) {
        const uint32_t id = kn[a];
        int l = 0, h = nfv;
        while (l < h) {
            const int mid = (l + h) >> 1;
            if (fn[mid] < id) l = mid + 1; else h = mid;
        }
        if (l < nfv && fn[l] == id) shared_nodes[atomicAdd(&n_shared, 1)] = make_int2(a, l);
    }
    __syncthreads();
    const int32_t* ks = K.fv_start + (size_t)kf * (K.cap + 1);
    const int32_t* fs = F.fv_start + (size_t)fr * (F.cap + 1);
    const int32_t* kfeat = K.fv_features + (size_t)kf * K.cap;
    const int32_t* ffeat = F.fv_features + (size_t)fr * F.cap;
    const uint4* kdesc = reinterpret_cast<const uint4*>(K.desc + (size_t)kf * K.cap * 32);
    const uint4* fdesc = reinterpret_cast<const uint4*>(F.desc + (size_t)fr * F.cap * 32);
    const uint8_t* has = K.has_point + (size_t)kf * K.cap;
    const spslam_keypoint* kk = K.keys + (size_t)kf * K.cap;
    const spslam_keypoint* fk = F.keys + (size_t)fr * F.cap;
    const float factor = 1.0f / kHisto;
    int count = 0;
    for (int s = wave; s < n_shared; s += kThreads / 64) {
        const int2 nd = shared_nodes[s];
        const int f0 = fs[nd.y], f1 = fs[nd.y + 1];
        for (int q = ks[nd.x]; q < ks[nd.x + 1]; q++) {
            const int ikf = kfeat[q];
            if (!has[ikf]) continue;
            const uint4 a0 = kdesc[2 * ikf], a1 = kdesc[2 * ikf + 1];
            Best b{256, 1 << 30, 256};
            for (int r = f0 + lane; r < f1; r += 64) {
                const int jf = ffeat[r];
                if (bin[jf] != -1) continue;  // vpMapPointMatches[realIdxF] already set
                const int d = hamming(a0, a1, fdesc[2 * jf], fdesc[2 * jf + 1]);
                if (d < b.b1) { b.b2 = b.b1; b.b1 = d; b.i1 = r; }
                else if (d < b.b2) b.b2 = d;
            }
#pragma unroll
            for (int o = 1; o < 64; o <<= 1) {
                Best x{__shfl_xor(b.b1, o), __shfl_xor(b.i1, o), __shfl_xor(b.b2, o)};
                b = merge(b, x);
            }
            if (b.b1 <= kThLow && (float)b.b1 < __fmul_rn(nn_ratio, (float)b.b2)) {
                const int jf = ffeat[b.i1];
                int bn = 0;
                if (check_ori) {
                    float rot = __fsub_rn(kk[ikf].angle, fk[jf].angle);
                    if (rot < 0.0f) rot = __fadd_rn(rot, 360.0f);
                    bn = (int)roundf(__fmul_rn(rot, factor));
                    if (bn == kHisto) bn = 0;
                }
                if (lane == 0) {
                    match[jf] = ikf;
                    bin[jf] = (signed char)bn;
                    if (check_ori) atomicAdd(&hist[bn], 1);
                }
                count++;
            }
            __builtin_amdgcn_wave_barrier();
        }
    }
    if (lane == 0 && count) atomicAdd(&n_total, count);
    __syncthreads();
    if (check_ori) {
        if (t == 0) three_maxima(hist, &ind[0], &ind[1], &ind[2]);
        __syncthreads();
        int removed = 0;
        for (int i = t; i < nF; i += kThreads) {
            const int bn = bin[i];
            if (bn >= 0 && bn != ind[0] && bn != ind[1] && bn != ind[2]) {
                match[i] = -1;
                removed++;
            }
        }
        if (removed) atomicAdd(&n_removed, removed);
        __syncthreads();
    }
    int32_t* mo = match_out + (size_t)p * F.cap;
    for (int i = t; i < nF; i += kThreads) mo[i] = match[i];
    if (t == 0) nmatches_out[p] = n_total - n_removed;
}

}  // namespace bow

hipError_t bow_transform_launch(const VocabDev& V, int n_frames, const uint8_t* desc, const int* counts, int cap,
                                int levelsup, uint32_t* s_word, double* s_weight, uint32_t* s_node,
                                const BowOut& out, hipStream_t s, KernelTimer* timer) {
    if (n_frames < 1 || cap < 1 || V.n_nodes < 2) return hipErrorInvalidValue;
    int P = 64;
    while (P < cap) P <<= 1;
    if (P > 8192) return hipErrorInvalidValue;  // 128 KB of LDS keys + values
    // dynamic LDS beyond the default 64 KB needs the per-kernel opt-in (set once)
    static const hipError_t lds_attr = hipFuncSetAttribute((const void*)bow::bow_vectors_kernel,
                                                           hipFuncAttributeMaxDynamicSharedMemorySize, 8192 * 16);
    if (lds_attr != hipSuccess) return lds_attr;
    const int tf = V.weighting == 0 || V.weighting == 1;  // TF_IDF, TF
    const int must = V.scoring != 5;                       // all but DOT_PRODUCT normalise
    const int l2 = V.scoring == 1;
    const long long n = (long long)n_frames * cap;
    if (timer) timer->begin(kKindBowWords, s);
    hipLaunchKernelGGL(bow::bow_words_kernel, dim3((unsigned)((n + bow::kThreads - 1) / bow::kThreads)),
                       dim3(bow::kThreads), 0, s, V, desc, counts, cap, n_frames, V.L - levelsup, s_word, s_weight,
                       s_node);
    if (timer) timer->end(kKindBowWords, s);
    if (timer) timer->begin(kKindBowVectors, s);
    hipLaunchKernelGGL(bow::bow_vectors_kernel, dim3(n_frames), dim3(bow::kThreads), (size_t)P * 16, s, cap, P, tf,
                       must, l2, counts, s_word, s_weight, s_node, out);
    if (timer) timer->end(kKindBowVectors, s);
    return hipGetLastError();
}

hipError_t bow_search_launch(int n_pairs, const int2* pairs, const BowSide& kf, const BowSide& fr, float nn_ratio,
                             int check_ori, int32_t* match, int* nmatches, hipStream_t s, KernelTimer* timer) {
    if (n_pairs < 1 || kf.cap < 1 || fr.cap < 1) return hipErrorInvalidValue;
    const size_t lds = (size_t)fr.cap * 4 + (size_t)kf.cap * 8 + (size_t)fr.cap;
    if (lds > 150 * 1024) return hipErrorInvalidValue;
    static const hipError_t lds_attr = hipFuncSetAttribute((const void*)bow::bow_search_kernel,
                                                           hipFuncAttributeMaxDynamicSharedMemorySize, 150 * 1024);
    if (lds_attr != hipSuccess) return lds_attr;
    if (timer) timer->begin(kKindBowMatch, s);
    hipLaunchKernelGGL(bow::bow_search_kernel, dim3(n_pairs), dim3(bow::kThreads), (lds + 15) / 16 * 16, s, pairs, kf,
                       fr, nn_ratio, check_ori, match, nmatches);
    if (timer) timer->end(kKindBowMatch, s);
    return hipGetLastError();
}

}  // namespace spslam
