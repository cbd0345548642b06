#include "rsa_seed.h"
void seed_bufs_release(SeedBufs& b) {
    for (int i = 0; i < 24; ++i) if (b.p[i]) (void)hipFree(b.p[i]);
    for (int i = 0; i < 8; ++i) if (b.h[i]) (void)hipHostFree(b.h[i]);
}
extern "C" int rsa_randstrobes(rsa_ctx*, const rsa_read_batch*, rsa_randstrobe_batch*) { return RSA_ERR_ARG; }
extern "C" int rsa_seed(rsa_ctx*, const rsa_read_batch*, int32_t, uint32_t, rsa_nam_batch*) { return RSA_ERR_ARG; }
