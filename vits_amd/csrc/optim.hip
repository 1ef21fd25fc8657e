// optim.hip — fused RAdam step for the discriminator optimizer of the
// train_stft step (train_stft.py:97: `RAdam(net_d.parameters(), 1e-4)`,
// radam.py:35-99, the LiyuanLucasLiu rectified Adam).
//
// One launch updates every parameter tensor (the tensor list travels in the
// kernel arguments, up to VITS_RADAM_MAX per launch), with GradScaler's skip
// rule built in: when *found_inf != 0 nothing is touched (torch/amp
// grad_scaler.py step()).  The step count and the rectification scalars live
// on the device, so the step needs no host sync and can be graph-captured.
// Arithmetic per element follows radam.py:
//   v = b2 v + (1-b2) g^2 ; m = b1 m + (1-b1) g ; t += 1
//   N = Nmax - 2 t b2^t / (1 - b2^t),  Nmax = 2/(1-b2) - 1
//   N >= 5: p -= lr * s * m / (sqrt(v) + eps),
//           s = sqrt((1-b2^t)(N-4)/(Nmax-4)(N-2)/N Nmax/(Nmax-2)) / (1-b1^t)
//   N <  5: p -= lr * m / (1-b1^t)
// (weight decay: p -= wd * lr * p first, radam.py:87-88; coupled into p,
// not an L2 term on g).  The scalars are
// computed in double precision as the reference's Python floats are.
#include "common.h"

namespace {

struct RadamList {
  vits_radam_tensor t[VITS_RADAM_MAX];
};

// scal[0] = step count t (float), scal[1] = skip flag, scal[2] = lr * s,
// scal[3] = 1 if N >= 5, scal[4] = gradient multiplier (1 / grad_scale),
// scal[5] = weight_decay * lr.  lr comes from lr_dev (a device double that an
// lr scheduler updates in place, so a captured step sees every change) when
// given, else from the launch argument.
__global__ void radam_scalars_kernel(float* __restrict__ scal, const float* __restrict__ found_inf,
                                     const float* __restrict__ grad_scale, double lr_arg,
                                     const double* __restrict__ lr_dev, double beta1, double beta2,
                                     double weight_decay) {
  if (threadIdx.x != 0 || blockIdx.x != 0) return;
  const bool skip = found_inf && *found_inf != 0.f;
  scal[1] = skip ? 1.f : 0.f;
  scal[4] = grad_scale ? 1.0f / *grad_scale : 1.0f;
  if (skip) return;
  const double lr = lr_dev ? *lr_dev : lr_arg;
  const double t = (double)scal[0] + 1.0;
  scal[0] = (float)t;
  const double b2t = pow(beta2, t);
  const double nmax = 2.0 / (1.0 - beta2) - 1.0;
  const double n = nmax - 2.0 * t * b2t / (1.0 - b2t);
  double s;
  if (n >= 5.0)
    s = sqrt((1.0 - b2t) * (n - 4.0) / (nmax - 4.0) * (n - 2.0) / n * nmax / (nmax - 2.0)) /
        (1.0 - pow(beta1, t));
  else
    s = 1.0 / (1.0 - pow(beta1, t));
  scal[2] = (float)(lr * s);
  scal[3] = n >= 5.0 ? 1.f : 0.f;
  scal[5] = (float)(weight_decay * lr);
}

__global__ __launch_bounds__(256) void radam_update_kernel(const RadamList list,
                                                          const float* __restrict__ scal,
                                                          float beta1, float beta2, float omb1,
                                                          float omb2, float eps) {
  if (scal[1] != 0.f) return;  // GradScaler skip
  const vits_radam_tensor& T = list.t[blockIdx.y];
  const float step = scal[2];
  const bool rect = scal[3] != 0.f;
  const float gmul = scal[4];
  const float wd_lr = scal[5];
  for (int64_t i = blockIdx.x * 256 + threadIdx.x; i < T.numel; i += (int64_t)gridDim.x * 256) {
    const float g = gmul == 1.0f ? T.grad[i] : T.grad[i] * gmul;
    float v = T.exp_avg_sq[i];
    float m = T.exp_avg[i];
    v = v * beta2 + omb2 * g * g;  // exp_avg_sq.mul_(b2).addcmul_(g, g, value=1-b2)
    m = m * beta1 + omb1 * g;      // exp_avg.mul_(b1).add_(g, alpha=1-b1)
    T.exp_avg_sq[i] = v;
    T.exp_avg[i] = m;
    float p = T.param[i];
    if (wd_lr != 0.f) p = p - wd_lr * p;
    p = rect ? p - step * (m / (sqrtf(v) + eps)) : p - step * m;  // addcdiv_ / add_
    T.param[i] = p;
  }
}

}  // namespace

extern "C" int vits_radam_step(const vits_radam_tensor* tensors, int n, float* scal,
                               const float* found_inf, const float* grad_scale, double lr,
                               const double* lr_dev, double beta1, double beta2, double eps, double weight_decay,
                               void* stream) {
  VITS_CHECK_ARG(tensors && scal && n >= 0);
  hipStream_t s = as_stream(stream);
  hipLaunchKernelGGL(radam_scalars_kernel, dim3(1), dim3(64), 0, s, scal, found_inf, grad_scale,
                     lr, lr_dev, beta1, beta2, weight_decay);
  int rc = vits_launch_status();
  if (rc) return rc;
  for (int base = 0; base < n; base += VITS_RADAM_MAX) {
    const int cnt = n - base < VITS_RADAM_MAX ? n - base : VITS_RADAM_MAX;
    RadamList list;
    int64_t most = 1;
    for (int i = 0; i < cnt; ++i) {
      list.t[i] = tensors[base + i];
      VITS_CHECK_ARG(list.t[i].param && list.t[i].grad && list.t[i].exp_avg && list.t[i].exp_avg_sq);
      if (list.t[i].numel > most) most = list.t[i].numel;
    }
    const int64_t want = (most + 255) / 256;
    const int bx = (int)(want < 64 ? want : 64);
    hipLaunchKernelGGL(radam_update_kernel, dim3(bx, cnt), dim3(256), 0, s, list, scal,
                       (float)beta1, (float)beta2, (float)(1.0 - beta1), (float)(1.0 - beta2),
                       (float)eps);
    rc = vits_launch_status();
    if (rc) return rc;
  }
  return VITS_OK;
}
