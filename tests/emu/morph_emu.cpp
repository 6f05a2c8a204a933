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
