// Diagnostic only: batch reset, then one env's map-generation scratch (placed pieces, piece
// transforms, bounds, flags) as the device left it.
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -Iinclude -Igym-eldorado_amd/csrc tools/dbg_gen.cpp -o tools/dbg_gen
//   tools/dbg_gen N BASE DIFF ENV...
#include "../gym-eldorado_amd/csrc/cog_engine.hip"
#include "../gym-eldorado_amd/csrc/cog_abi.cpp"
#include <cstdio>

int main(int argc, char **argv) {
  const size_t n = strtoul(argv[1], nullptr, 10);
  const uint32_t base = (uint32_t)strtoul(argv[2], nullptr, 10);
  const int diff = atoi(argv[3]);
  cog_env *env;
  if (cog_env_create(n, 0, &env) || cog_env_reset(env, base, 4, 3, diff, 100000, 0)) {
    printf("setup failed: %s\n", cog_last_error());
    return 1;
  }
  const cog::DevState &s = env->sh[0].s;
  for (int a = 4; a < argc; a++) {
    const size_t i = strtoul(argv[a], nullptr, 10);
    cog::GenScratch g;
    cog::EnvPriv pv;
    if (hipMemcpy(&g, s.gen + i, sizeof g, hipMemcpyDeviceToHost) != hipSuccess ||
        hipMemcpy(&pv, s.priv + i, sizeof pv, hipMemcpyDeviceToHost) != hipSuccess)
      return 1;
    printf("env %zu: pieces", i);
    for (int k = 0; k < g.npieces; k++) printf(" %d", g.pieces[k]);
    printf("  bounds %d %d %d %d dims %d %d flags %#x\n  tf:", pv.minx, pv.miny, pv.maxx, pv.maxy, pv.dimx, pv.dimy, pv.flags);
    for (int q = 0; q < COG_N_PIECES; q++)
      if (g.pcx[q] || g.pcy[q] || g.prot[q]) printf(" %d:[%d,%d,%d]", q, g.pcx[q], g.pcy[q], g.prot[q]);
    printf("\n");
  }
  return 0;
}
