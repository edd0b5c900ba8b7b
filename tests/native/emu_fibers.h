// Fiber scheduler of the host wave emulator (test infrastructure): every GPU thread of a workgroup is a fiber of one
// host thread; hd.h (SM_HOST_EMU) turns wave64 operations and __syncthreads into barriers of a wave's / the
// workgroup's fibers, which emu_launch runs until they reach one. One translation unit per emulated kernel library
// includes this file once, after the kernel header.
#pragma once
#include <cstdio>
#include <cstdlib>
#include <functional>
#include <memory>
#include <vector>

sm_dim3 threadIdx, blockIdx, gridDim, blockDim;
unsigned long long (*sm_emu::wave_buf)[64] = nullptr;

// ---- fibers: a minimal x86-64 (System V) context switch; callee-saved registers live on the fiber's own stack
extern "C" void sm_fiber_switch(void** save_sp, void* load_sp);
asm(R"(
.text
.globl sm_fiber_switch
.type sm_fiber_switch,@function
sm_fiber_switch:
  pushq %rbp
  pushq %rbx
  pushq %r12
  pushq %r13
  pushq %r14
  pushq %r15
  movq %rsp, (%rdi)
  movq %rsi, %rsp
  popq %r15
  popq %r14
  popq %r13
  popq %r12
  popq %rbx
  popq %rbp
  ret
.size sm_fiber_switch, .-sm_fiber_switch
)");

namespace {

constexpr size_t kFiberStack = 256 << 10;

struct Fiber {
  void* sp = nullptr;
  std::unique_ptr<char[]> stack;
  bool done = false;
  unsigned waiting = 0;  // 0: runnable; else the generation of the barrier it waits on + 1
  int group = -1;        // -1: block barrier, else its wave
};

struct Sched {
  std::vector<Fiber> f;
  void* main_sp = nullptr;
  int cur = -1;
  std::function<void()> body;
  // barriers: arrivals and generation of the block barrier and of each wave's
  int block_arrived = 0;
  unsigned block_gen = 0;
  std::vector<int> wave_arrived;
  std::vector<unsigned> wave_gen;
};
Sched* g_s = nullptr;

void yield_to_main() { sm_fiber_switch(&g_s->f[g_s->cur].sp, g_s->main_sp); }

[[noreturn]] void fiber_entry() {
  g_s->body();
  g_s->f[g_s->cur].done = true;
  yield_to_main();
  abort();  // a finished fiber is never resumed
}

void* init_stack(Fiber& fb) {
  fb.stack.reset(new char[kFiberStack]);
  uintptr_t top = ((uintptr_t)fb.stack.get() + kFiberStack) & ~(uintptr_t)15;
  void** p = (void**)top;
  *--p = nullptr;                   // alignment slot: rsp % 16 == 8 at fiber_entry, as after a call
  *--p = (void*)&fiber_entry;       // popped by `ret`
  for (int k = 0; k < 6; ++k) *--p = nullptr;  // rbp rbx r12 r13 r14 r15
  return (void*)p;
}

template <typename F>
void emu_launch(int grid, int block, F body) {
  gridDim.x = (unsigned)grid;
  blockDim.x = (unsigned)block;
  const int nw = block / 64;
  std::unique_ptr<unsigned long long[][64]> bufs(new unsigned long long[nw][64]);
  sm_emu::wave_buf = bufs.get();
  for (int b = 0; b < grid; ++b) {
    Sched s;
    s.f.resize(block);
    s.body = body;
    s.wave_arrived.assign(nw, 0);
    s.wave_gen.assign(nw, 0);
    for (auto& fb : s.f) fb.sp = init_stack(fb);
    g_s = &s;
    blockIdx.x = (unsigned)b;
    for (;;) {
      int live = 0, ran = 0;
      for (int t = 0; t < block; ++t) {
        Fiber& fb = s.f[t];
        if (fb.done) continue;
        ++live;
        if (fb.waiting) {
          const unsigned g = fb.group < 0 ? s.block_gen : s.wave_gen[fb.group];
          if (g + 1 == fb.waiting) continue;  // its barrier has not opened yet
          fb.waiting = 0;
        }
        s.cur = t;
        threadIdx.x = (unsigned)t;
        sm_fiber_switch(&s.main_sp, fb.sp);
        ++ran;
      }
      if (!live) break;
      if (!ran) {
        fprintf(stderr, "wave emulator: deadlock (every live fiber waits on a barrier)\n");
        abort();
      }
    }
    g_s = nullptr;
  }
}

void arrive(int group, int size, int& arrived, unsigned& gen) {
  Fiber& fb = g_s->f[g_s->cur];
  if (++arrived == size) {  // the last one opens the barrier and goes on
    arrived = 0;
    ++gen;
    return;
  }
  fb.group = group;
  fb.waiting = gen + 1;
  yield_to_main();
}

}  // namespace

void sm_emu::wave_sync() {
  const int w = (int)(threadIdx.x >> 6);
  arrive(w, 64, g_s->wave_arrived[w], g_s->wave_gen[w]);
}
void sm_emu::block_sync() { arrive(-1, (int)blockDim.x, g_s->block_arrived, g_s->block_gen); }

