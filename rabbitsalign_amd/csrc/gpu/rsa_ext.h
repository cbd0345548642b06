// rsa_ext.h -- host/device shared descriptors of the extension kernels.
#pragma once
#include <stdint.h>
#include "../../../include/rsa_gpu.h"

struct ExtJobDev {
    uint64_t q_off;    // into the device query buffer
    uint64_t r_off;    // absolute offset into the device reference (contig start + window start)
    uint32_t qlen, rlen;
    uint64_t cig_off;  // CIGAR slot (qlen + rlen + 8 entries) in the device pool
};

struct ScanRes {
    int score1, ref_end1, read_end1, ref_begin1, read_begin1, flag, word, status;
};

#define RSA_RAW_CAP (1024 + 2048 + 16)
