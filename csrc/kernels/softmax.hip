// Softmax, fused softmax + multinomial cross-entropy (SoftmaxWithLoss) and top-k
// accuracy over rows of a [M, C] bf16 matrix (channels contiguous: for NHWC 4-D
// inputs every pixel is a row).
//
// Reference: SoftmaxLayer (5 kernels: channel_max/subtract/exp/sum/div,
// caffe/src/caffe/layers/softmax_layer.cu:13-139), SoftmaxLossForwardGPU/BackwardGPU
// (softmax_loss_layer.cu:11-124) followed by two cublasSasum host syncs, and the
// CPU-only AccuracyLayer (accuracy_layer.cpp) which forced a D2H copy.
// Here: one wave per row (fp32 math, 64-lane shuffles), a deterministic second pass for
// the scalar loss / normaliser, everything stays on the device.
#include "common.h"

#define FLT_MIN_ 1.175494351e-38f

// one wave per row: prob row (fp32), per-row nll and valid flag
__global__ void softmax_xent_fwd(const bf16_t* __restrict__ x, const float* __restrict__ labels,
                                 float* __restrict__ prob, float* __restrict__ row_loss, float* __restrict__ row_valid,
                                 int M, int C, int has_ignore, int ignore_label) {
  const int lane = threadIdx.x & 63;
  const int row = blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
  if (row >= M) return;
  const bf16_t* xr = x + (long long)row * C;
  float m = -INFINITY;
  for (int c = lane; c < C; c += 64) m = fmaxf(m, bf2f(xr[c]));
  m = wave_max(m);
  float s = 0.f;
  for (int c = lane; c < C; c += 64) s += __expf(bf2f(xr[c]) - m);
  s = wave_sum(s);
  const float inv = 1.f / s;
  float* pr = prob + (long long)row * C;
  for (int c = lane; c < C; c += 64) pr[c] = __expf(bf2f(xr[c]) - m) * inv;
  if (lane == 0) {
    int lab = (int)labels[row];
    bool valid = !(has_ignore && lab == ignore_label);
    float nll = 0.f;
    if (valid) {
      float p = __expf(bf2f(xr[min(max(lab, 0), C - 1)]) - m) * inv;
      nll = -__logf(fmaxf(p, FLT_MIN_));
    }
    row_loss[row] = nll;
    row_valid[row] = valid ? 1.f : 0.f;
  }
}

// loss = sum(row_loss) / max(norm, 1) where norm = sum(row_valid) (normalize) or outer_num
__global__ void xent_reduce(const float* __restrict__ row_loss, const float* __restrict__ row_valid, int M,
                            int normalize, float outer_num, float* __restrict__ out_loss, float* __restrict__ out_norm) {
  __shared__ float ls[16], vs[16];
  float l = 0.f, v = 0.f;
  for (int i = threadIdx.x; i < M; i += blockDim.x) {
    l += row_loss[i];
    v += row_valid[i];
  }
  l = wave_sum(l);
  v = wave_sum(v);
  if ((threadIdx.x & 63) == 0) {
    ls[threadIdx.x >> 6] = l;
    vs[threadIdx.x >> 6] = v;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    float L = 0.f, V = 0.f;
    for (int w = 0; w < (int)(blockDim.x >> 6); ++w) { L += ls[w]; V += vs[w]; }
    float norm = normalize ? V : outer_num;
    norm = fmaxf(norm, 1.f);
    out_loss[0] = L / norm;
    out_norm[0] = norm;
  }
}

extern "C" int sn_softmax_xent_fwd(const bf16_t* x, const float* labels, float* prob, float* row_loss,
                                   float* row_valid, float* out_loss, float* out_norm, long long M, long long C,
                                   long long has_ignore, long long ignore_label, long long normalize,
                                   long long outer_num, hipStream_t st) {
  const int rows_per_block = 4;
  hipLaunchKernelGGL(softmax_xent_fwd, dim3((unsigned)((M + rows_per_block - 1) / rows_per_block)), dim3(256), 0, st, x,
                     labels, prob, row_loss, row_valid, (int)M, (int)C, (int)has_ignore, (int)ignore_label);
  hipLaunchKernelGGL(xent_reduce, dim3(1), dim3(1024), 0, st, row_loss, row_valid, (int)M, (int)normalize,
                     (float)outer_num, out_loss, out_norm);
  return SN_CHECK_LAUNCH();
}

// dx = (prob - onehot(label)) * valid * loss_weight / norm
__global__ void softmax_xent_bwd(const float* __restrict__ prob, const float* __restrict__ labels,
                                 const float* __restrict__ loss_weight, const float* __restrict__ norm,
                                 bf16_t* __restrict__ dx, int M, int C, int has_ignore, int ignore_label) {
  const long long total = (long long)M * C;
  const float scale = loss_weight[0] / norm[0];
  for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < total; i += (long long)gridDim.x * blockDim.x) {
    const int row = (int)(i / C), c = (int)(i - (long long)row * C);
    const int lab = (int)labels[row];
    float g = 0.f;
    if (!(has_ignore && lab == ignore_label)) g = (prob[i] - (c == lab ? 1.f : 0.f)) * scale;
    dx[i] = f2bf(g);
  }
}

extern "C" int sn_softmax_xent_bwd(const float* prob, const float* labels, const float* loss_weight, const float* norm,
                                   bf16_t* dx, long long M, long long C, long long has_ignore, long long ignore_label,
                                   hipStream_t st) {
  hipLaunchKernelGGL(softmax_xent_bwd, dim3(sn_blocks(M * C, 256, 16384)), dim3(256), 0, st, prob, labels, loss_weight,
                     norm, dx, (int)M, (int)C, (int)has_ignore, (int)ignore_label);
  return SN_CHECK_LAUNCH();
}

// plain softmax (bf16 in/out, fp32 math), one wave per row
__global__ void softmax_fwd(const bf16_t* __restrict__ x, bf16_t* __restrict__ y, int M, int C) {
  const int lane = threadIdx.x & 63;
  const int row = blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
  if (row >= M) return;
  const bf16_t* xr = x + (long long)row * C;
  float m = -INFINITY;
  for (int c = lane; c < C; c += 64) m = fmaxf(m, bf2f(xr[c]));
  m = wave_max(m);
  float s = 0.f;
  for (int c = lane; c < C; c += 64) s += __expf(bf2f(xr[c]) - m);
  s = wave_sum(s);
  const float inv = 1.f / s;
  for (int c = lane; c < C; c += 64) y[(long long)row * C + c] = f2bf(__expf(bf2f(xr[c]) - m) * inv);
}

// dx = y * (dy - sum(dy*y))
__global__ void softmax_bwd(const bf16_t* __restrict__ dy, const bf16_t* __restrict__ y, bf16_t* __restrict__ dx,
                            int M, int C) {
  const int lane = threadIdx.x & 63;
  const int row = blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
  if (row >= M) return;
  const long long b = (long long)row * C;
  float d = 0.f;
  for (int c = lane; c < C; c += 64) d += bf2f(dy[b + c]) * bf2f(y[b + c]);
  d = wave_sum(d);
  for (int c = lane; c < C; c += 64) dx[b + c] = f2bf(bf2f(y[b + c]) * (bf2f(dy[b + c]) - d));
}

extern "C" int sn_softmax_fwd(const bf16_t* x, bf16_t* y, long long M, long long C, hipStream_t st) {
  hipLaunchKernelGGL(softmax_fwd, dim3((unsigned)((M + 3) / 4)), dim3(256), 0, st, x, y, (int)M, (int)C);
  return SN_CHECK_LAUNCH();
}

extern "C" int sn_softmax_bwd(const bf16_t* dy, const bf16_t* y, bf16_t* dx, long long M, long long C, hipStream_t st) {
  hipLaunchKernelGGL(softmax_bwd, dim3((unsigned)((M + 3) / 4)), dim3(256), 0, st, dy, y, dx, (int)M, (int)C);
  return SN_CHECK_LAUNCH();
}

// top-k accuracy: hit if fewer than k classes score strictly higher than the label
__global__ void accuracy_rows(const bf16_t* __restrict__ x, const float* __restrict__ labels, float* __restrict__ hit,
                              float* __restrict__ valid, int M, int C, int k, int has_ignore, int ignore_label) {
  const int lane = threadIdx.x & 63;
  const int row = blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
  if (row >= M) return;
  const int lab = (int)labels[row];
  const bf16_t* xr = x + (long long)row * C;
  const float ls = bf2f(xr[min(max(lab, 0), C - 1)]);
  float cnt = 0.f;
  for (int c = lane; c < C; c += 64) cnt += bf2f(xr[c]) > ls ? 1.f : 0.f;
  cnt = wave_sum(cnt);
  if (lane == 0) {
    bool v = !(has_ignore && lab == ignore_label);
    hit[row] = (v && cnt < (float)k) ? 1.f : 0.f;
    valid[row] = v ? 1.f : 0.f;
  }
}

extern "C" int sn_accuracy(const bf16_t* x, const float* labels, float* hit, float* valid, float* out_acc,
                           float* out_norm, long long M, long long C, long long k, long long has_ignore,
                           long long ignore_label, hipStream_t st) {
  hipLaunchKernelGGL(accuracy_rows, dim3((unsigned)((M + 3) / 4)), dim3(256), 0, st, x, labels, hit, valid, (int)M,
                     (int)C, (int)k, (int)has_ignore, (int)ignore_label);
  hipLaunchKernelGGL(xent_reduce, dim3(1), dim3(1024), 0, st, hit, valid, (int)M, 1, (float)M, out_acc, out_norm);
  return SN_CHECK_LAUNCH();
}
