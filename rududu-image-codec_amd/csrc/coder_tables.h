// coder_tables.h -- format constants of the serial coder, one copy shared by
// the reference-shaped coder (entropy.cpp), the record encoder (encoder.cpp)
// and the register decoder (decoder.cpp).  Transcribed from the reference;
// they are part of the .ric bitstream contract.
#pragma once
#include <cstdint>

namespace ric {
namespace tables {

// CBitCodec::thres, src/lib/bitcodec.cpp:40-42
inline constexpr uint16_t kBitThres[11] = {2584, 1512, 745, 371, 185, 92, 46, 23, 12, 6, 3};
// CGeomCodec::thres, K, shift: src/lib/geomcodec.cpp:44-54; entry 24 of K /
// shift guards an index the reference never reaches on valid data
inline constexpr uint16_t kGeoThres[11] = {1512, 2584, 3351, 3725, 3911, 4004, 4050, 4073, 4084, 4090, 4093};
inline constexpr uint8_t kGeoK[25] = {0,0,0,0,0,0,0,0,0,0,1,2,3,4,5,6,7,8,9,10,11,12,13,14,14};
inline constexpr uint8_t kGeoShift[25] = {10,9,8,7,6,5,4,3,2,1,1,1,1,1,1,1,1,1,1,1,1,1,1,1,1};
// CMuxCodec::CnkLen / CnkLost, src/lib/muxcodec.cpp:294-332
inline constexpr uint8_t kCnkLen[16][8] = {
	{0,0,0,0,0,0,0,0},{1,0,0,0,0,0,0,0},{2,2,0,0,0,0,0,0},{2,3,2,0,0,0,0,0},
	{3,4,4,3,0,0,0,0},{3,4,5,4,3,0,0,0},{3,5,6,6,5,3,0,0},{3,5,6,7,6,5,3,0},
	{4,6,7,7,7,7,6,4},{4,6,7,8,8,8,7,6},{4,6,8,9,9,9,9,8},{4,7,8,9,10,10,10,9},
	{4,7,9,10,11,11,11,11},{4,7,9,10,11,12,12,12},{4,7,9,11,12,13,13,13},{4,7,10,11,13,13,14,14}};
inline constexpr uint16_t kCnkLost[16][8] = {
	{0,0,0,0,0,0,0,0},{0,0,0,0,0,0,0,0},{1,1,0,0,0,0,0,0},{0,2,0,0,0,0,0,0},
	{3,6,6,3,0,0,0,0},{2,1,12,1,2,0,0,0},{1,11,29,29,11,1,0,0},{0,4,8,58,8,4,0,0},
	{7,28,44,2,2,44,28,7},{6,19,8,46,4,46,8,19},{5,9,91,182,50,50,182,91},
	{4,62,36,17,232,100,232,17},{3,50,226,309,761,332,332,761},{2,37,148,23,46,1093,664,1093},
	{1,23,57,683,1093,3187,1757,1757},{0,8,464,228,3824,184,4944,3514}};
// the edge block's geometric context, src/lib/bandcodec.cpp:409-423
inline constexpr uint8_t kKConv2[9][16] = {
	{15}, {7,15}, {4,10,15}, {3,7,11,15}, {2,4,7,10,12,15}, {1,3,5,7,9,11,13,15},
	{1,3,4,6,8,10,11,13,15}, {0,2,3,4,6,7,8,10,11,12,14,15},
	{0,1,2,3,4,5,6,7,8,9,10,11,12,13,14,15}};
inline constexpr uint8_t kKConv1[16] = {0,1,2,3,0,4,0,5,6,0,0,7,0,0,0,8};

}  // namespace tables
}  // namespace ric
