// oracle/ref_video.cpp -- TEST INFRASTRUCTURE ONLY (the checker of the video
// path).  Linked with the reference library compiled in place from
// /root/reference/src/lib by oracle/Makefile into oracle/_ref/ricvid_ref.
//
// The reference video codec is CRududuCodec (src/lib/rududucodec.cpp): EPZS
// motion search (COBME, obme.cpp), OBMC (COBMC, obmc.cpp) with adaptive
// Huffman MV coding (CHuffCodec, huffcodec.cpp), quarter-pel planes
// (CImageBuffer::calc_sub, imagebuffer.cpp:90-121; CImage::interH/interV,
// image.cpp:280-342) and the 3-level wavelet closed loop over CWavelet2D.
// As written, rududucodec.cpp:74 and :83 pass each plane's START to
// CWavelet2D::TransformI, which since ric_0.2 takes the END pointer
// (wavelet2d.cpp:507: the output starts DimY rows before it; ric.cpp:216-225
// passes the end).  The reconstruction then lands DimY rows above the plane,
// outside the allocation for plane 0: the reference video codec crashes on its
// first frame (ASan: wavelet2d.cpp:514 via rududucodec.cpp:74).
//
// This driver therefore restates CRududuCodec's 80 lines of orchestration
// (rududucodec.cpp:32-141: the constructor, quants(), encodeImage,
// decodeImage, encode, decode) line for line, with the one change of passing
// the plane's end pointer to TransformI, and calls the reference's own
// CImageBuffer, CImage, COBME, COBMC, CWavelet2D and CMuxCodec for everything
// else.  CImage's planes and COBMC's vectors are private; the driver reads them
// through member pointers obtained by explicit template instantiation (the
// access rules do not apply there), to dump them.
//
// Uninitialised memory: CImage::Init allocates with new[] and never clears
// (image.cpp:60), and calc_sub reads one sample outside each plane before
// extend() writes the borders (image.cpp:290-296, 322-328): the reference
// reads whatever the allocator returned -- zeros from a fresh mmap at video
// sizes.  The driver pins that to zeros at every size: its global operator
// new hands out fresh zeroed pages (below).
//
//   ricvid_ref W H Q NFRAMES in.rgb out.bin
//     in.rgb : NFRAMES x 3 planes R, G, B of H rows x W bytes, bottom row
//              first (CImage::inputSGI, image.cpp:96-123, stride W)
//     out.bin: per frame: u32 size (encode()'s return), the size + 2 stream
//              bytes, the encoder's output image (3 x H x W int16: Y, Co, Cg),
//              u32 decode()'s return, the decoder's output image, the
//              encoder's motion vectors ((W >> 3) x (H >> 3) u32), and the
//              bordered planes of the encoder's output image (3 x (H + 30) x
//              (W + 30) int16, rows and columns -15 .. +14 past the edges),
//              and that image as CImage::outputYV12<char, false>(pOut, W,
//              -128) writes it (W * H * 3 / 2 bytes, testmotion.cpp:62)
#include <chrono>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <new>
#include <vector>

#include <sys/mman.h>
#include <unistd.h>

#include "imagebuffer.h"
#include "muxcodec.h"
#include "obme.h"
#include "wavelet2d.h"

// ------------------------------------------- zeroed, ILP32-mirrored memory
// The video classes index with unsigned int arithmetic that goes "negative":
// CImage::interH reads in[i - 1] at i = 0 (image.cpp:290, 293, 296; i is
// unsigned int), COBME::EPZS and COBMC::encode/decode read pCurMV[i - dimX]
// and pCurMV[i - dimX + 1] (obme.cpp:194-200, obmc.cpp:364-366, 412-414; i,
// dimX unsigned int).  On the 32-bit targets the code was written for, the
// wrapped index is the element just before; with 64-bit pointers it is
// 2^32 elements AFTER (the reference segfaults: ASan, image.cpp:290).
// Every allocation here is a memfd mapped at p and mirrored at p + 4, 8 and
// 16 GiB (2^32 elements of 1, 2, 4 bytes), so those reads land on exactly the
// element the 32-bit build reads -- the reference's own code runs unmodified
// with its ILP32 semantics.  Fresh pages are zero (see above).
namespace {
const size_t kPage = 4096, kGiB = (size_t)1 << 30;
const size_t kMirror[3] = {4 * kGiB, 8 * kGiB, 16 * kGiB};
const uint64_t kMagic = 0x52494356494431ull;   // "RICVID1"
struct Hdr { uint64_t magic, reserve, size, pad; };

void* mirrored_alloc(size_t n)
{
	const size_t len = (n + sizeof(Hdr) + kPage - 1) / kPage * kPage;
	const size_t reserve = kMirror[2] + len;
	char* base = (char*)mmap(nullptr, reserve, PROT_NONE, MAP_PRIVATE | MAP_ANONYMOUS | MAP_NORESERVE, -1, 0);
	if (base == MAP_FAILED) return nullptr;
	const int fd = memfd_create("ricvid", 0);
	if (fd < 0 || ftruncate(fd, (off_t)len) != 0) { munmap(base, reserve); return nullptr; }
	bool ok = mmap(base, len, PROT_READ | PROT_WRITE, MAP_SHARED | MAP_FIXED, fd, 0) != MAP_FAILED;
	for (size_t m : kMirror)
		ok = ok && mmap(base + m, len, PROT_READ | PROT_WRITE, MAP_SHARED | MAP_FIXED, fd, 0) != MAP_FAILED;
	close(fd);
	if (!ok) { munmap(base, reserve); return nullptr; }
	// the header sits just before the user block, inside the first page
	char* p = base + len - ((n + 15) & ~(size_t)15);
	p -= (uintptr_t)p % 64;
	if (p < base + sizeof(Hdr)) p = base + sizeof(Hdr);
	Hdr* h = (Hdr*)p - 1;
	h->magic = kMagic; h->reserve = reserve; h->size = (size_t)((char*)p - base);
	return p;
}
}  // namespace

void* operator new(size_t n)
{
	void* p = mirrored_alloc(n ? n : 1);
	if (!p) throw std::bad_alloc();
	return p;
}
void* operator new[](size_t n) { return operator new(n); }
void operator delete(void* p) noexcept
{
	if (!p) return;
	Hdr* h = (Hdr*)p - 1;
	if (h->magic != kMagic) abort();
	munmap((char*)p - h->size, h->reserve);
}
void operator delete[](void* p) noexcept { operator delete(p); }
void operator delete(void* p, size_t) noexcept { operator delete(p); }
void operator delete[](void* p, size_t) noexcept { operator delete(p); }

using namespace rududu;

// --------------------------------------------- private member access (dumps)
template <class Tag> struct Member { static typename Tag::type ptr; };
template <class Tag> typename Tag::type Member<Tag>::ptr;
template <class Tag, typename Tag::type P> struct Take {
	struct Init { Init() { Member<Tag>::ptr = P; } };
	static Init init;
};
template <class Tag, typename Tag::type P> typename Take<Tag, P>::Init Take<Tag, P>::init;

struct ImgPlanes { typedef short* (CImage::*type)[MAX_COMPONENT]; };
struct ImgAlign { typedef unsigned int CImage::*type; };
struct MvField { typedef sMotionVector* COBMC::*type; };
template struct Take<ImgPlanes, &CImage::pImage>;
template struct Take<ImgAlign, &CImage::dimXAlign>;
template struct Take<MvField, &COBMC::pMV>;

static short* plane(CImage* im, int c) { return (im->*Member<ImgPlanes>::ptr)[c]; }
static int align_of(CImage* im) { return (int)(im->*Member<ImgAlign>::ptr); }

// ------------------------------------ CRududuCodec (rududucodec.cpp:26-141)
#define WAV_LEVELS 3
#define TRANSFORM cdf97
#define BUFFER_SIZE (SUB_IMAGE_CNT + 1)

class VideoCodec {
public:
	int quant;
	VideoCodec(cmode mode, int width, int height, int component)
		: quant(0), images(width, height, component, BUFFER_SIZE), predImage(0), codec(0, 0), key_count(0),
		  w(width), h(height)
	{
		wavelet = new CWavelet2D(width, height, WAV_LEVELS);
		wavelet->SetWeight(TRANSFORM);
		if (mode == rududu::encode) {
			obmc = (COBMC*)new COBME(width >> 3, height >> 3);
			predImage = new CImage(width, height, component, ALIGN);
		} else {
			obmc = new COBMC(width >> 3, height >> 3);
			predImage = new CImage(width, height, component, ALIGN);
		}
	}
	~VideoCodec()
	{
		delete predImage;
		delete obmc;
		delete wavelet;
	}
	static short quants(int idx)
	{
		static const unsigned short Q[5] = {32768, 37641, 43238, 49667, 57052};
		if (idx == 0) return 0;
		idx--;
		int r = 10 - idx / 5;
		return (short)((Q[idx % 5] + (1 << (r - 1))) >> r);
	}
	// the one change: TransformI gets the plane's end pointer
	void encodeImage(CImage* pImage)
	{
		const int S = align_of(pImage);
		dump(pImage, "res");
		for (int c = 0; c < 3; c++) {
			wavelet->Transform(plane(pImage, c), S, TRANSFORM);
			wavelet->CodeBand(&codec, quants(quant + 20), quants(quant + 12));
			wavelet->TSUQi(quants(quant + 20));
			wavelet->TransformI(plane(pImage, c) + (long)h * S, S, TRANSFORM);
		}
	}
	void decodeImage(CImage* pImage)
	{
		const int S = align_of(pImage);
		for (int c = 0; c < 3; c++) {
			wavelet->DecodeBand(&codec);
			wavelet->TSUQi(quants(quant + 20));
			wavelet->TransformI(plane(pImage, c) + (long)h * S, S, TRANSFORM);
		}
	}
	int encode(unsigned char* pImage, int stride, unsigned char* pBuffer, CImage** outImage)
	{
		codec.initCoder(0, pBuffer);
		images.insert(0);
		images[0][0]->inputSGI(pImage, stride, -128);
		if (key_count != 0) {
			COBME* obme = (COBME*)obmc;
			images.calc_sub(1);
			obme->EPZS(images);
			obme->encode(&codec);
			obme->apply_mv(images, *predImage);
			dump(predImage, "pred");
			*images[0][0] -= *predImage;
			encodeImage(images[0][0]);
			*images[0][0] += *predImage;
			pBuffer[0] |= 0x80;
		} else {
			encodeImage(images[0][0]);
		}
		key_count++;
		if (key_count == 10) key_count = 0;
		frame++;
		*outImage = images[0][0];
		images.remove(1);
		return codec.endCoding() - pBuffer - 2;
	}
	int decode(unsigned char* pBuffer, CImage** outImage)
	{
		codec.initDecoder(pBuffer);
		images.insert(0);
		if (pBuffer[0] & 0x80) {
			images.calc_sub(1);
			obmc->decode(&codec);
			obmc->apply_mv(images, *predImage);
			decodeImage(images[0][0]);
			*images[0][0] += *predImage;
		} else {
			decodeImage(images[0][0]);
		}
		*outImage = images[0][0];
		images.remove(1);
		return codec.getSize();
	}
	const sMotionVector* mvs() const { return obmc->*Member<MvField>::ptr; }
	// diagnostics: RICVID_DUMP=<dir> writes every frame's residual planes (the
	// encoder's image as encodeImage receives it) and prediction, bordered
	int frame = 0;
	void dump(CImage* im, const char* what)
	{
		const char* dir = getenv("RICVID_DUMP");
		if (!dir) return;
		char path[4096];
		snprintf(path, sizeof path, "%s/%s_f%d.i16", dir, what, frame);
		FILE* f = fopen(path, "wb");
		if (!f) return;
		const int S = align_of(im);
		for (int c = 0; c < 3; c++)
			for (int y = -15; y < h + 15; y++) fwrite(plane(im, c) + (long)y * S - 15, 2, w + 30, f);
		fclose(f);
	}

private:
	CImageBuffer images;
	CImage* predImage;
	COBMC* obmc;
	CWavelet2D* wavelet;
	CMuxCodec codec;
	int key_count;
	int w, h;
};

static void put_planes(FILE* f, CImage* im, int w, int h, int border)
{
	const int S = align_of(im);
	for (int c = 0; c < 3; c++)
		for (int y = -border; y < h + border; y++)
			fwrite(plane(im, c) + (long)y * S - border, 2, w + 2 * border, f);
}

int main(int argc, char** argv)
{
	if (argc != 7) {
		fprintf(stderr, "usage: %s W H Q NFRAMES in.rgb out.bin\n", argv[0]);
		return 2;
	}
	const int W = atoi(argv[1]), H = atoi(argv[2]), Q = atoi(argv[3]), N = atoi(argv[4]);
	FILE* fi = fopen(argv[5], "rb");
	FILE* fo = fopen(argv[6], "wb");
	if (!fi || !fo || W < 16 || H < 16) return 2;
	VideoCodec enc(rududu::encode, W, H, 3), dec(rududu::decode, W, H, 3);
	enc.quant = Q;
	dec.quant = Q;
	const size_t fsz = (size_t)W * H * 3;
	std::vector<unsigned char> frame(fsz), buf(fsz * 4 + 4096), dbuf(fsz * 4 + 4096);
	// RICVID_TIME set: the encode and decode calls' wall time on stderr (the
	// video bench's CPU baseline, scripts/video_bench.py)
	const bool timed = getenv("RICVID_TIME") != nullptr;
	double t_enc = 0, t_dec = 0;
	for (int k = 0; k < N; k++) {
		if (fread(frame.data(), 1, fsz, fi) != fsz) return 3;
		std::fill(buf.begin(), buf.end(), 0);
		CImage* out = 0;
		auto t0 = std::chrono::steady_clock::now();
		const int size = enc.encode(frame.data(), W, buf.data(), &out);
		t_enc += std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
		const uint32_t s32 = (uint32_t)size;
		fwrite(&s32, 4, 1, fo);
		fwrite(buf.data(), 1, size + 2, fo);
		put_planes(fo, out, W, H, 0);
		CImage* eout = out;
		// the decoder reads exactly the stream, zero padded
		std::fill(dbuf.begin(), dbuf.end(), 0);
		memcpy(dbuf.data(), buf.data(), size + 2);
		CImage* dout = 0;
		t0 = std::chrono::steady_clock::now();
		const uint32_t d32 = (uint32_t)dec.decode(dbuf.data(), &dout);
		t_dec += std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
		fwrite(&d32, 4, 1, fo);
		put_planes(fo, dout, W, H, 0);
		fwrite(enc.mvs(), 4, (size_t)(W >> 3) * (H >> 3), fo);
		put_planes(fo, eout, W, H, 15);
		// CImage::outputYV12<char, false>(pOut, W, -128) of the encoder's
		// image, as testmotion.cpp:62 writes it (image.cpp:148-185)
		// (odd sizes: outputYV12 writes a little past W * H * 3 / 2)
		std::vector<char> yv((size_t)W * H * 3 / 2 + 4 * (size_t)W + 64, 0);
		eout->outputYV12<char, false>(yv.data(), W, -128);
		fwrite(yv.data(), 1, (size_t)W * H * 3 / 2, fo);
	}
	fclose(fo);
	fclose(fi);
	if (timed) fprintf(stderr, "{\"frames\": %d, \"encode_s\": %.6f, \"decode_s\": %.6f}\n", N, t_enc, t_dec);
	return 0;
}
