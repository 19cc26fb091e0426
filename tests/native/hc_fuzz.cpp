// hc_fuzz.cpp -- the product's host decoder (csrc/entropy.cpp, decoder.cpp)
// on untrusted .ric bytes, built with AddressSanitizer + UndefinedBehavior-
// Sanitizer (tests/native/Makefile hc_fuzz).  For every .ric file given: the
// full stream, every 1/16 prefix (truncation), bit-flipped variants and
// random payloads of the same geometry.  Any sanitizer report aborts with a
// non-zero status; a clean run prints "ok N".
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <iterator>
#include <random>
#include <vector>

extern "C" long hc_decode(const uint8_t* in, long len, int nplanes, int w, int h, int levels, int lc,
                          int32_t* bands_out, double* secs);

static long total_bands(int w, int h, int levels)
{
	long n = 0;
	int lw = w, lh = h, lev = levels;
	for (;;) {
		n += (long)((lw + 1) >> 1) * ((lh + 1) >> 1) + (long)(lw >> 1) * ((lh + 1) >> 1) + (long)((lw + 1) >> 1) * (lh >> 1);
		if (!(lev > 1 && lw > 15 && lh > 15)) break;
		lw >>= 1; lh >>= 1; lev--;
	}
	return n + (long)(lw >> 1) * (lh >> 1);
}

#include <chrono>
static void run(const std::vector<uint8_t>& ric, int w, int h, int c, std::vector<int32_t>& out)
{
	static const bool verbose = getenv("HC_FUZZ_VERBOSE") != nullptr;
	const auto t0 = std::chrono::steady_clock::now();
	// the decoder input: two zero bytes, then the payload (src/ric/ric.cpp:203-205)
	std::vector<uint8_t> buf(2 + (ric.size() > 9 ? ric.size() - 9 : 0), 0);
	if (ric.size() > 9) memcpy(buf.data() + 2, ric.data() + 9, ric.size() - 9);
	hc_decode(buf.data(), (long)buf.size(), c, w, h, 5, 1, out.data(), nullptr);
	if (verbose)
		fprintf(stderr, "%zu bytes %.3f s\n", ric.size(),
		        std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count());
}

int main(int argc, char** argv)
{
	std::mt19937 rng(12345);
	long runs = 0;
	for (int a = 1; a < argc; a++) {
		std::ifstream f(argv[a], std::ios::binary);
		std::vector<uint8_t> ric((std::istreambuf_iterator<char>(f)), std::istreambuf_iterator<char>());
		if (ric.size() < 9 || memcmp(ric.data(), "RUD2", 4) != 0) { fprintf(stderr, "bad file %s\n", argv[a]); return 1; }
		const int w = ric[4] | (ric[5] << 8), h = ric[6] | (ric[7] << 8), c = ((ric[8] >> 5) & 1) ? 3 : 1;
		std::vector<int32_t> out((size_t)total_bands(w, h, 5) * c + 16);
		run(ric, w, h, c, out);
		runs++;
		for (int k = 0; k < 16; k++) {                     // truncations
			std::vector<uint8_t> t(ric.begin(), ric.begin() + 9 + (ric.size() - 9) * k / 16);
			run(t, w, h, c, out);
			runs++;
		}
		for (int k = 0; k < 48; k++) {                     // bit flips
			std::vector<uint8_t> t = ric;
			for (int j = 0; j <= k % 4; j++) {
				const size_t pos = 9 + rng() % (t.size() - 9);
				t[pos] ^= (uint8_t)(1u << (rng() % 8));
			}
			run(t, w, h, c, out);
			runs++;
		}
		for (int k = 0; k < 16; k++) {                     // garbage payloads
			std::vector<uint8_t> t(ric.begin(), ric.begin() + 9);
			const size_t n = 1 + rng() % (2 * (ric.size() - 9) + 64);
			for (size_t j = 0; j < n; j++) t.push_back((uint8_t)rng());
			run(t, w, h, c, out);
			runs++;
		}
	}
	printf("ok %ld\n", runs);
	return 0;
}
