// hc_main.cpp -- development tool: times the product's host coder (record
// encoder + band decoder, via tests/native/host_coder_harness.cpp) on a C3
// stage-1 band dump.  Usage: hc_main DUMP REPS.  Prints one line per rep.
#include <cstdio>
#include <cstdlib>
#include <vector>
#include <cstdint>
extern "C" long hc_encode_rec(const int32_t*, long, int, int, int, int, int, uint8_t*, long, double*, double*);
extern "C" long hc_decode(const uint8_t*, long, int, int, int, int, int, int32_t*, double*);
int main(int argc, char** argv)
{
	if (argc < 2) return 2;
	FILE* f = fopen(argv[1], "rb");
	if (!f) return 1;
	fseek(f, 0, SEEK_END);
	long n = ftell(f) / 4;
	fseek(f, 0, SEEK_SET);
	std::vector<int32_t> b(n);
	if (fread(b.data(), 4, n, f) != (size_t)n) return 1;
	fclose(f);
	long cap = 7680L * 4320 * 4 + 4096;
	std::vector<uint8_t> out(cap);
	std::vector<int32_t> dec(n);
	int reps = argc > 2 ? atoi(argv[2]) : 3;
	for (int r = 0; r < reps; r++) {
		double s1, s2, s3;
		long len = hc_encode_rec(b.data(), n, 1, 7680, 4320, 5, 1, out.data(), cap, &s1, &s2);
		hc_decode(out.data(), len, 1, 7680, 4320, 5, 1, dec.data(), &s3);
		uint64_t h = 1469598103934665603ull;              // FNV-1a of the decoded bands
		for (long i = 0; i < n; i++) h = (h ^ (uint32_t)dec[i]) * 1099511628211ull;
		printf("len %ld enc %.2f dec %.2f hash %016llx\n", len, s1 * 1e3, s3 * 1e3, (unsigned long long)h);
	}
	return 0;
}
