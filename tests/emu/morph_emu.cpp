// Host emulation of the gfx950 morph kernel (TEST TOOL, never shipped).
// Compiles the very same mcaq_morph.h with g++ and runs morph_image() with a
// single "thread", so tests can compare the kernel's arithmetic with the
// numpy oracle on CPU.  Built by tests/emu/build_emu.py.
#define MCAQ_NO_HIP 1
#include <stdlib.h>
#include <string.h>
#include <vector>
#include "../../mcaq_yolo_amd/csrc/mcaq_morph.h"

extern "C" int emu_morph(const mcaq_morph_scale* s) {
  using namespace mcaq;
  const int NT = s->ht * s->wt;
  std::vector<char> planes(plane_bytes(s->Hc, s->Wc) + 64), shm(fixed_bytes() + tile_bytes(NT) + 64);
  std::vector<char> tshm(tiles_lds_bytes(s->H, s->W, NT) + 64);
  for (int b = 0; b < s->B; ++b) {
    Ctx ctx{0, 1};
    if (s->flags & F_PHI) {
      for (int role = 0; role < 2; ++role) {   // edge and mask workgroups
        Planes pl; Shared sh;
        carve_planes(planes.data(), s->Hc, s->Wc, pl);
        carve_shared(shm.data(), sh);
        if (s->flags & F_CANNY_LEGACY) morph_edges<true>(ctx, *s, b, role, pl, sh);
        else morph_edges<false>(ctx, *s, b, role, pl, sh);
      }
    }
    Shared sh2;
    carve_shared(tshm.data(), sh2);
    morph_tiles(ctx, *s, b, sh2, nullptr, 0, 1, nullptr);
  }
  return 0;
}

// pass A in band mode (mcaq_band.h): every band of an image, then its edge
// workgroup, then pass B as above.  s->pwork must hold
// band_work_bytes(B, Hc, Wc, tile) bytes.
extern "C" int emu_morph_band(const mcaq_morph_scale* s) {
  using namespace mcaq;
  if (!band_eligible(*s)) return 1;
  const int NT = s->ht * s->wt;
  std::vector<char> blds(band_lds_bytes(s->Wc, s->tile) + 64), elds(edge_lds_bytes(s->Hc, s->Wc) + 64);
  std::vector<char> tshm(tiles_lds_bytes(s->H, s->W, NT) + 64);
  const int nb = band_count(s->Hc, s->tile);
  Ctx ctx{0, 1};
  for (int b = 0; b < s->B; ++b)
    for (int k = 0; k < nb; ++k) band_pass(ctx, *s, b, k, blds.data());
  for (int b = 0; b < s->B; ++b) edge_image(ctx, *s, b, elds.data());
  for (int b = 0; b < s->B; ++b) {
    Shared sh2;
    carve_shared(tshm.data(), sh2);
    morph_tiles(ctx, *s, b, sh2, nullptr, 0, 1, nullptr);
  }
  return 0;
}

// pass B as the batch-wide tile kernels (mcaq_tiles_batch.h) after the
// per-image pass A: the same per-tile functions in the kernels' order, the
// MLPs in their scalar forms (the device MFMA blocks equal them).  Tile
// intermediates go through the free tile_tmp slots, as on the device.
extern "C" int emu_morph_tb(const mcaq_morph_scale* s) {
  using namespace mcaq;
  if (!tiles_batch_eligible(*s)) return 1;
  const int NT = s->ht * s->wt, n = s->B * NT;
  std::vector<char> planes(plane_bytes(s->Hc, s->Wc) + 64), shm(fixed_bytes() + tile_bytes(NT) + 64);
  Ctx ctx{0, 1};
  for (int b = 0; b < s->B; ++b)
    for (int role = 0; role < 2; ++role) {
      Planes pl; Shared sh;
      carve_planes(planes.data(), s->Hc, s->Wc, pl);
      carve_shared(shm.data(), sh);
      morph_edges<false>(ctx, *s, b, role, pl, sh);
    }
  float* tt = s->tile_tmp;
  for (int u = 0; u < n; ++u) {   // head
    const int b = u / NT, t = u - b * NT;
    float p[8];
    phi_of_tile(*s, b, t, tt + (size_t)u * TT_STRIDE, p);
    if (s->phi_out) for (int k = 0; k < 8; ++k) s->phi_out[(size_t)u * 8 + k] = p[k];
    const float c = complexity_mlp_tile(s->cmlp, p);
    tt[(size_t)u * TT_STRIDE + TT_CRAW] = c;
    if (s->cmlp_out) s->cmlp_out[u] = c;
  }
  for (int u = 0; u < n; ++u) {   // map
    const int b = u / NT, t = u - b * NT, th = t / s->wt, tw = t - th * s->wt;
    const float* crow = tt + (size_t)b * NT * TT_STRIDE + TT_CRAW;
    const float c = bilateral_tile(t, th, tw, s->ht, s->wt, NT, [&](int k) { return crow[(size_t)k * TT_STRIDE]; });
    if (s->c_out) s->c_out[u] = c;
    if (s->flags & F_SOFTMASK)
      tt[(size_t)u * TT_STRIDE + TT_ACT] = act_tile(s->absmean + (size_t)b * s->H * s->W, s->H, s->W, s->ht, s->wt, th, tw);
    const float bv = finish_bits(mapper_mlp_tile(s->mapper, c, s->min_bits, s->max_bits), *s);
    tt[(size_t)u * TT_STRIDE + TT_BITS] = bv;
    if (s->bits_out) s->bits_out[u] = bv;
  }
  if (s->flags & F_SOFTMASK)
    for (int u = 0; u < n; ++u) {   // mask
      const int b = u / NT, t = u - b * NT, th = t / s->wt, tw = t - th * s->wt;
      const float* row = tt + (size_t)b * NT * TT_STRIDE;
      float amax = -3.402823466e38f;
      for (int j = 0; j < NT; ++j) amax = fmaxp(amax, row[(size_t)j * TT_STRIDE + TT_ACT]);
      const float den = amax + 1e-8f;
      const bool vl = aten_softmax_vec_lane((long long)(s->batch_offset + b) * NT + t, (long long)s->batch_total * NT,
                                            NT, s->softmax_threads);
      const float mtv = smask_tile(
          s->smask, th, tw, s->ht, s->wt,
          [&](int q) { return clampf_((row[(size_t)q * TT_STRIDE + TT_BITS] - 2.0f) / 6.0f, 0.0f, 1.0f); },
          [&](int q) { return row[(size_t)q * TT_STRIDE + TT_ACT] / den; }, vl);
      if (s->mt_out) s->mt_out[u] = mtv;
    }
  if ((s->flags & F_SOFTMASK) && s->m_out)
    for (int b = 0; b < s->B; ++b)
      for (int h = 0; h < s->H; ++h)
        for (int w = 0; w < s->W; ++w)
          s->m_out[((size_t)b * s->H + h) * s->W + w] = mplane_pixel(s->mt_out + (size_t)b * NT, s->H, s->W, s->ht, s->wt, h, w);
  return 0;
}
