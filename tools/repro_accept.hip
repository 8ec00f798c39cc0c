// Repro: device log_alpha / accept on fixed inputs vs the host.
#pragma clang fp contract(off)
#include <hip/hip_runtime.h>
#include <cstdio>
#include "../mcmc-in-tonga_amd/csrc/chain_logic.h"

// the pre-fix shape of log_alpha: a switch whose default returns -dphi
__host__ __device__ double log_alpha_switch(const tdchain::Params &P, const tdchain::Proposal &p, double phi,
                                            double phi_n, double czeta, double zk, double zn, const double *lnN) {
    const double dphi = (phi_n - phi) / (2.0 * P.temperature);
    switch (p.action) {
        case tdchain::kBirth: {
            const double dz = czeta - p.zeta;
            return ((lnN[1] - lnN[2]) + P.log_prior_birth) + ((dz * dz) / (2.0 * P.sig_zeta * P.sig_zeta) - dphi);
        }
        case tdchain::kDeath: {
            const double dz = zk - zn;
            return ((lnN[1] - lnN[0]) + P.log_prior_death) + (-(dz * dz) / (2.0 * P.sig_zeta * P.sig_zeta) - dphi);
        }
        default:
            return -dphi;
    }
}

__global__ void k(const tdchain::Params *P, const tdchain::Proposal *p, const double *in, double *out) {
    __shared__ double ln[3];
    if (threadIdx.x < 3) ln[threadIdx.x] = in[5 + threadIdx.x];
    __syncthreads();
    if (threadIdx.x == 0) {
        const tdchain::Proposal pp = *p;
        out[0] = tdchain::log_alpha(*P, pp, in[0], in[1], in[2], in[3], in[4], ln);
        out[2] = log_alpha_switch(*P, pp, in[0], in[1], in[2], in[3], in[4], ln);
        out[1] = tdchain::accept(*P, pp, in[0], in[1], in[2], in[3], in[4], ln) ? 1.0 : 0.0;
    }
}

int main() {
    tdchain::Params P{};
    P.temperature = 1.0;
    P.sig_zeta = 5.0;
    P.zeta_scale = 50.0;
    P.log_prior_birth = -1.38365;
    P.log_prior_death = 1.38365;
    double in[9] = {13830.735098345343, 13790.554010674889, 0.0, 40.2154, 0.0, 5.29832, 5.3033, 5.30827, 201};
    for (int act = 1; act <= 4; ++act) {
        tdchain::Proposal p{};
        p.action = act; p.active = 1; p.valid = 1; p.zeta = 40.2154;
        p.u_accept = 0.28477480029180763; p.log_u = -1.2560565854805521;
        tdchain::Params *dP; tdchain::Proposal *dp; double *din, *dout;
        hipMalloc(&dP, sizeof P); hipMalloc(&dp, sizeof p); hipMalloc(&din, sizeof in); hipMalloc(&dout, 24);
        hipMemcpy(dP, &P, sizeof P, hipMemcpyHostToDevice);
        hipMemcpy(dp, &p, sizeof p, hipMemcpyHostToDevice);
        hipMemcpy(din, in, sizeof in, hipMemcpyHostToDevice);
        hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, dP, dp, din, dout);
        double o[3];
        hipMemcpy(o, dout, 24, hipMemcpyDeviceToHost);
        const double h = tdchain::log_alpha(P, p, in[0], in[1], in[2], in[3], in[4], in + 5);
        const double hs = log_alpha_switch(P, p, in[0], in[1], in[2], in[3], in[4], in + 5);
        printf("act %d device la %.17g acc %g switch %.17g | host la %.17g switch %.17g\n", act, o[0], o[1], o[2], h, hs);
    }
    return 0;
}
