// example_decode.cpp -- how a VTM-style host drives the MM path through the C++ shim.
//
//   make -C vvc-extension-mm_amd example   (hipcc: the example allocates its planes with hipMalloc)
//
// Builds a 256x128 ERP sequence context with the MPA models, uploads two synthetic reference
// pictures, reprojects one block (MVReprojection call shape) and predicts a picture's PU list
// four times -- host list (mm_pred), device-resident list (mm_pred_device) and two pictures in one
// launch chain (mm_pred_device_multi) -- and checks that all predictions agree.  The sequence
// parameters come from an SPS MM fragment written and parsed back (mm360::MMSyntax), and the PUs'
// motion models make a CABAC motion_model() round trip.  Exit 0 and "OK" on success; exit 2 when no
// HIP device is present.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <vector>

#include "mm360_vtm.hpp"

int main() {
  const int W = 256, H = 128;
  try {
    // the SPS as an encoder writes it and a decoder parses it (VLCWriter.cpp:1110-1142 /
    // VLCReader.cpp:1920-1980): MPA on, MMOffset4x4 code 1, ERP projection
    mm_sps_mm sps{};
    sps.mpa = 1;
    sps.mm_offset_4x4 = 1;
    sps.ged_flavor = 1;
    sps.projection_fct = 2;
    std::vector<uint8_t> rbsp;
    int64_t wpos = 5;  // inside a larger SPS: any bit offset
    mm360::MMSyntax::writeSPS(sps, rbsp, wpos);
    int64_t rpos = 5;
    const mm_sps_mm parsed = mm360::MMSyntax::readSPS(rbsp.data(), wpos, rpos);
    if (rpos != wpos || parsed.mpa != 1 || parsed.mm_offset_4x4 != 1) return 1;
    const mm_seq_params prm = mm360::MMSyntax::seqParams(parsed, W, H, 1, 10, 128, 128);
    if (prm.active_models != ((1u << MM_CLASSIC) | (1u << MM_MPA_FRONT_BACK) | (1u << MM_MPA_LEFT_RIGHT) |
                              (1u << MM_MPA_TOP_BOTTOM)))
      return 1;
    mm360::Context ctx(prm, 0);
    std::vector<int16_t> y(W * H), c((W / 2) * (H / 2));
    for (int poc : {0, 16}) {
      for (int i = 0; i < W * H; i++) y[i] = (int16_t)((i * 7 + poc * 13) % 1024);
      for (int i = 0; i < (W / 2) * (H / 2); i++) c[i] = (int16_t)((i * 5 + poc) % 1024);
      ctx.uploadReference(poc, y.data(), W, c.data(), c.data(), W / 2, false);
    }
    mm360::MVReprojectionGPU rep;
    rep.init(&ctx);
    mm360::FixedPair f = rep.reprojectMotionVectorSubblocks(32, 16, 16, 8, 37, -21, MM_MPA_FRONT_BACK, 0, 8, 0);
    if (f.rows != 2 || f.cols != 4) return 1;

    // MM-MVP per candidate, as the merge / AMVP builders call it in decoding order
    // (MVReprojection::motionVectorInDesiredMotionModel -> mm_mvp_convert_host), timed per call
    const int32_t e1[3] = {1 << 24, 0, 0};
    ctx.setEpipole(8, -1, e1);
    const int n_calls = 20000;
    long mv_sum = 0;
    const auto t0 = std::chrono::steady_clock::now();
    for (int i = 0; i < n_calls; i++) {
      const int m0 = MM_MPA_FRONT_BACK + i % 3, m1 = MM_MPA_FRONT_BACK + (i / 3) % 3;
      const auto mv = rep.motionVectorInDesiredMotionModel(4 * (i % 60) + 2, 4 * ((i / 60) % 30) + 2, 37 + i % 50,
                                                           -21 + i % 40, m0, m1, 4, 4, 8, 0, 8, 16, 16 * (i % 14), 16,
                                                           16, 16, 16 * (i % 14) + 16, 16, 16, 16);
      mv_sum += mv.first + mv.second;
    }
    const double us = std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count() / n_calls;

    mm360::InterPredictionMM pred(&ctx);
    for (int by = 0; by < H; by += 16)
      for (int bx = 0; bx < W; bx += 16) {
        const int mv[2][2] = {{(bx * 3) % 97 - 48, (by * 5) % 61 - 30}, {17, -9}};
        const int ref[2] = {0, (bx / 16) % 2 ? 16 : -1};
        const int model[2] = {MM_MPA_FRONT_BACK + (bx / 16) % 3, MM_MPA_TOP_BOTTOM};
        pred.addPU(bx, by, 16, 16, mv, ref, model);
      }
    // the PUs' motion_model() through CABAC and back (CABACWriter / CABACReader::motion_model,
    // m_mmCodingDepth 9, m_mmPredType 0 as the apps set them)
    {
      const std::vector<int32_t> act = mm360::MMSyntax::activeModels(parsed);
      const std::vector<mm_pu_desc>& pus = pred.pus();
      std::vector<int32_t> cand(pus.size() * MM_NUM_MODEL_IDS, -1), models(pus.size()), back(pus.size());
      for (size_t i = 0; i < pus.size(); i++) {
        std::copy(act.begin(), act.end(), cand.begin() + i * MM_NUM_MODEL_IDS);
        models[i] = pus[i].model[0];
      }
      std::vector<uint8_t> stream(64 + 4 * pus.size());
      int64_t nbytes = 0;
      mm360::check(nullptr, mm_motion_model_encode(&parsed, 32, 0, 9, (int)pus.size(), cand.data(), nullptr, models.data(),
                                                   stream.data(), (int64_t)stream.size(), &nbytes),
                   "mm_motion_model_encode");
      mm360::check(nullptr, mm_motion_model_decode(&parsed, 32, 0, 9, (int)pus.size(), cand.data(), nullptr, stream.data(),
                                                   nbytes, back.data()),
                   "mm_motion_model_decode");
      if (back != models) return 1;
    }
    int16_t *dy[4], *dc[4][2];
    for (int k = 0; k < 4; k++) {
      if (hipMalloc(&dy[k], W * H * 2) != hipSuccess || hipMalloc(&dc[k][0], W * H / 2) != hipSuccess ||
          hipMalloc(&dc[k][1], W * H / 2) != hipSuccess)
        return 1;
    }
    pred.predictPicture(8, dy[0], W, dc[0][0], dc[0][1], W / 2);

    // the same list from device memory
    mm_pu_desc* d_pus = nullptr;
    const std::vector<mm_pu_desc>& host = pred.pus();
    const size_t n = host.size();
    if (hipMalloc(&d_pus, n * sizeof(mm_pu_desc)) != hipSuccess) return 1;
    if (hipMemcpy(d_pus, host.data(), n * sizeof(mm_pu_desc), hipMemcpyHostToDevice) != hipSuccess) return 1;
    pred.predictPictureDevice(8, d_pus, (int)n, dy[1], W, dc[1][0], dc[1][1], W / 2);
    ctx.synchronize();

    // the same list twice in ONE launch chain (two independent pictures, mm_pred_device_multi)
    pred.predictPicturesDevice({mm_pic_job{8, d_pus, (int32_t)n, dy[2], W, dc[2][0], dc[2][1], W / 2},
                                mm_pic_job{8, d_pus, (int32_t)n, dy[3], W, dc[3][0], dc[3][1], W / 2}});
    ctx.synchronize();

    std::vector<int16_t> a(W * H), b(W * H);
    if (hipMemcpy(a.data(), dy[0], W * H * 2, hipMemcpyDeviceToHost) != hipSuccess) return 1;
    long sum = 0;
    for (int q = 1; q < 4; q++) {
      if (hipMemcpy(b.data(), dy[q], W * H * 2, hipMemcpyDeviceToHost) != hipSuccess) return 1;
      for (int k = 0; k < W * H; k++)
        if (a[k] != b[k]) {
          std::printf("MISMATCH picture %d at %d\n", q, k);
          return 1;
        }
    }
    for (int k = 0; k < W * H; k++) sum += a[k];
    std::printf("OK reproject(0,0)=(%d,%d) luma-sum=%ld\n", f.X(0, 0), f.Y(0, 0), sum);
    std::printf("MVP host per-call latency %.3f us (%d calls of motionVectorInDesiredMotionModel, MPA models, "
                "checksum %ld)\n", us, n_calls, mv_sum);
    for (int k = 0; k < 4; k++) {
      (void)hipFree(dy[k]);
      (void)hipFree(dc[k][0]);
      (void)hipFree(dc[k][1]);
    }
    (void)hipFree(d_pus);
    return 0;
  } catch (const mm360::Exception& e) {
    std::printf("mm360 error %d: %s\n", e.code(), e.what());
    return e.code() == MM_ERR_NODEV ? 2 : 1;
  }
}
