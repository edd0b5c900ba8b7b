// Query-specialised NFA kernels (nfa_jit.cpp): the NFA interpreter compiled per query plan with hiprtc.
#pragma once
#include <string>
#include <vector>

#include "kernels/nfa.h"
#include "kernels/primitives.h"

namespace sm {

// the JIT source for a plan blob (diagnostics / tests), with or without LDS staging of the key state
std::string nfa_jit_source(const std::vector<char>& blob, int compact = -1);
std::string nfa_jit_source(const std::vector<char>& blob, bool lds, int compact);
// target of the compile: the current device's gfx architecture, else the build's ARCH
std::string nfa_jit_arch();
// whether a batch of `records` query records runs the specialised kernel: env SM_NFA_JIT (0/1) wins, then the
// app option nfa_jit (0/1, -1 = automatic: batches of 2^20 records or more)
bool nfa_jit_wanted(int option, int64_t records);
// the code object of the plan's kernel (no device needed; throws with the compiler log on errors)
std::vector<char> nfa_jit_compile(const std::vector<char>& blob, int compact = -1);
// compiled kernel for this plan on the current device (cached per device and plan; throws on compile errors)
// compact: the batch's LaneEv form (0 / 1) compiled in as a constant; -1 = read from the batch at run time
void* nfa_jit_function(const std::vector<char>& blob, int compact = -1);
// dynamic LDS of the kernel (the staged per-key state words of a 64-lane workgroup; 0 when SM_NFA_JIT_LDS=0 or when
// they exceed the device's LDS per workgroup, in which case the kernel is built without the staging)
bool nfa_jit_lds();
int64_t nfa_jit_lds_bytes(const std::vector<char>& blob);
void launch_nfa_jit(void* fn, int64_t lds_bytes, const NfaBatch& b, int64_t* ks, int64_t* heap, int32_t heap_half,
                    int64_t lanes, int32_t nkeys, int32_t* err_dev, hipStream_t s);

}  // namespace sm
