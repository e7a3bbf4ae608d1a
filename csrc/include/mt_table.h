// Multi-tensor-apply launch table (host + device shared layout).
//
// Apex's engine (apex@f3a960f8:csrc/multi_tensor_apply.cuh) passes tensor
// addresses by value in a <4 KB kernel argument, which caps a launch at
// 110/64/48/36/30 tensors and 320 blocks, so a ResNet-50 optimizer step needs
// >= 5 launches and only ~1.25 blocks per CU on a 256-CU MI355X.
//
// Here the table lives in device memory instead: one TensorDesc per tensor and
// one ChunkDesc per kTile-element work unit.  A whole model fits in ONE launch
// with grid = #chunks (thousands of workgroups -> every CU busy), and the table
// is cached on the device keyed by the tensor addresses, so a steady-state
// optimizer step performs zero host->device metadata copies.
#pragma once
#include <stdint.h>

namespace amd {

constexpr int kMaxDepth = 6;
constexpr int kMTThreads = 256;                // 4 waves
constexpr int kMTUnroll = 4;                   // 8-element vectors per thread per tile
constexpr int kTile = kMTThreads * 8 * kMTUnroll;  // 8192 elements per workgroup

struct TensorDesc {
  void* ptr[kMaxDepth];
  int64_t numel;
  int32_t aligned;   // 1 if every pointer of this tensor is 16-byte aligned
  int32_t first_chunk;  // index of this tensor's first chunk in the chunk list
};

struct ChunkDesc {
  int32_t tensor;
  int32_t chunk;     // element offset = chunk * kTile
};

struct MTLaunch {
  const TensorDesc* tensors;   // device
  const ChunkDesc* chunks;     // device
  int32_t ntensors;
  int32_t nchunks;
};

}  // namespace amd
