// cgck_synth.hip — device-side synthetic batches and the
// streaming-read diagnostics probes.
#include "cgck_device.h"

namespace cgck {

// --------------------------------------------------------------------------
// Synthetic input: byte j of the stream = byte j&7 of
// splitmix64(seed, j>>3); then per-packet header stamps.
// --------------------------------------------------------------------------

__device__ __forceinline__ uint64_t splitmix64(uint64_t seed, uint64_t j)
{
	uint64_t z = seed + (j + 1) * 0x9e3779b97f4a7c15ull;
	z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ull;
	z = (z ^ (z >> 27)) * 0x94d049bb133111ebull;
	return z ^ (z >> 31);
}

__global__ __launch_bounds__(256) void synth_fill_kernel(uint8_t *base, uint64_t nbytes, uint64_t seed)
{
	const uint64_t nw = nbytes >> 3;
	uint64_t *w = reinterpret_cast<uint64_t *>(base);
	for (uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x; 2 * i < nw;
	     i += (uint64_t)gridDim.x * 256) {
		uint64_t j = 2 * i;
		if (j + 1 < nw) {
			ulonglong2 x = make_ulonglong2(splitmix64(seed, j), splitmix64(seed, j + 1));
			*reinterpret_cast<ulonglong2 *>(w + j) = x;
		} else {
			w[j] = splitmix64(seed, j);
		}
	}
	if (blockIdx.x == 0 && threadIdx.x < (nbytes & 7)) {
		uint64_t b = (nw << 3) + threadIdx.x;
		base[b] = (uint8_t)(splitmix64(seed, b >> 3) >> (8 * (b & 7)));
	}
}

__device__ __forceinline__ void stamp(uint8_t *ip, uint32_t len)
{
	ip[0] = 0x45;
	ip[1] = 0;
	ip[2] = (uint8_t)(len >> 8);
	ip[3] = (uint8_t)len;
	ip[9] = 6;
	ip[10] = 0;
	ip[11] = 0;
	if (len >= 38) {
		ip[36] = 0;
		ip[37] = 0;
	}
}

__global__ __launch_bounds__(256) void synth_stamp_strided_kernel(uint8_t *base, uint64_t n,
								  uint64_t stride, uint32_t len)
{
	for (uint64_t k = (uint64_t)blockIdx.x * 256 + threadIdx.x; k < n;
	     k += (uint64_t)gridDim.x * 256)
		stamp(base + k * stride, len);
}

__constant__ uint16_t c_imix_len[12] = {64, 576, 64, 64, 576, 64, 1500, 64, 576, 64, 64, 576};
__constant__ uint16_t c_imix_off[12] = {0, 64, 640, 704, 768, 1344, 1408, 2908, 2972, 3548, 3612, 3676};

__global__ __launch_bounds__(256) void synth_imix_kernel(uint8_t *base, uint32_t *desc, uint64_t n)
{
	for (uint64_t k = (uint64_t)blockIdx.x * 256 + threadIdx.x; k < n;
	     k += (uint64_t)gridDim.x * 256) {
		uint64_t off = (k / 12) * (uint64_t)kImixCycleBytes + c_imix_off[k % 12];
		uint32_t len = c_imix_len[k % 12];
		stamp(base + off, len);
		desc[3 * k + 0] = (uint32_t)off;
		desc[3 * k + 1] = (uint32_t)(off >> 32);
		desc[3 * k + 2] = len << 16; // l3_off 0, ip_len
	}
}

// The IMIX frames in ring slots: frame k (length of the 7:4:1 cycle) at
// k * stride + l3_off, e.g. the netmap layout (2048-byte slots, IPv4 at +14).
__global__ __launch_bounds__(256) void synth_ring_kernel(uint8_t *base, uint32_t *desc, uint64_t n, uint64_t stride,
							 uint32_t l3_off)
{
	for (uint64_t k = (uint64_t)blockIdx.x * 256 + threadIdx.x; k < n;
	     k += (uint64_t)gridDim.x * 256) {
		const uint64_t off = k * stride;
		const uint32_t len = c_imix_len[k % 12];
		stamp(base + off + l3_off, len);
		desc[3 * k + 0] = (uint32_t)off;
		desc[3 * k + 1] = (uint32_t)(off >> 32);
		desc[3 * k + 2] = (len << 16) | l3_off;
	}
}

hipError_t launch_synth_ring(uint8_t *base, uint32_t *desc, uint64_t n, uint64_t stride, uint32_t l3_off, int num_cus,
			     hipStream_t st)
{
	uint64_t want = (n + 255) / 256;
	int blocks = (int)(want < (uint64_t)num_cus * 8 ? want : (uint64_t)num_cus * 8);
	if (blocks < 1)
		blocks = 1;
	hipLaunchKernelGGL(synth_ring_kernel, dim3(blocks), dim3(256), 0, st, base, desc, n, stride, l3_off);
	return hipGetLastError();
}

hipError_t launch_synth_fill(uint8_t *base, uint64_t nbytes, uint64_t seed, int num_cus, hipStream_t st)
{
	uint64_t want = (nbytes / 16 + 255) / 256;
	int blocks = (int)(want < (uint64_t)num_cus * 8 ? want : (uint64_t)num_cus * 8);
	if (blocks < 1)
		blocks = 1;
	hipLaunchKernelGGL(synth_fill_kernel, dim3(blocks), dim3(256), 0, st, base, nbytes, seed);
	return hipGetLastError();
}

hipError_t launch_synth_stamp(uint8_t *base, uint64_t n, uint64_t stride, uint32_t len, int num_cus,
			      hipStream_t st)
{
	uint64_t want = (n + 255) / 256;
	int blocks = (int)(want < (uint64_t)num_cus * 8 ? want : (uint64_t)num_cus * 8);
	if (blocks < 1)
		blocks = 1;
	hipLaunchKernelGGL(synth_stamp_strided_kernel, dim3(blocks), dim3(256), 0, st, base, n, stride, len);
	return hipGetLastError();
}

hipError_t launch_synth_imix(uint8_t *base, uint32_t *desc, uint64_t n, int num_cus, hipStream_t st)
{
	uint64_t want = (n + 255) / 256;
	int blocks = (int)(want < (uint64_t)num_cus * 8 ? want : (uint64_t)num_cus * 8);
	if (blocks < 1)
		blocks = 1;
	hipLaunchKernelGGL(synth_imix_kernel, dim3(blocks), dim3(256), 0, st, base, desc, n);
	return hipGetLastError();
}

} // namespace cgck
