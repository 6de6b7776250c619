// Host cost of compiling one rank's collective (BuildSchedule) and planning it (PlanUnits), per call, for schedules
// from C5's smallest sizes to C3: what the per-communicator compiled-collective cache (executor.cc CompileCollective)
// saves on every repeated call.
//   g++ -O2 -Iinclude tools/compile_cost.cc -Lhccl_amd -lhccl_amd -Wl,-rpath,$PWD/hccl_amd -o /tmp/compile_cost
#include <chrono>
#include <cstdio>
#include <vector>
#include "hccl_amd.h"
int main(){
  struct C{int op,algo; unsigned n; unsigned long long cnt; HcclDataType dt;} cs[]={
   {0,4,8,512,HCCL_DATA_TYPE_FP16},{0,1,8,256,HCCL_DATA_TYPE_FP32},{0,2,8,1<<16,HCCL_DATA_TYPE_FP32},
   {0,3,8,1<<18,HCCL_DATA_TYPE_FP32},{0,8,8,1ull<<30,HCCL_DATA_TYPE_FP32},{0,3,8,1ull<<30,HCCL_DATA_TYPE_FP32}};
  for(auto&c:cs){
    std::vector<HcclAmdIrOp> ops(20000); uint64_t n=0,se=0; int32_t used=0;
    const int N=200; auto t0=std::chrono::steady_clock::now();
    for(int i=0;i<N;++i) HcclAmdBuildSchedule(c.op,c.algo,c.n,0,c.cnt,c.dt,0,0,ops.data(),ops.size(),&n,&used,&se);
    auto t1=std::chrono::steady_clock::now();
    uint64_t base[3]={1ull<<40,2ull<<40,3ull<<40}; std::vector<HcclAmdUnitPlan> u(20000); uint64_t nu=0;
    for(int i=0;i<N;++i) HcclAmdExecutorPlan(ops.data(),n,HcclAmdDataTypeSize(c.dt),base,u.data(),u.size(),&nu);
    auto t2=std::chrono::steady_clock::now();
    printf("algo %d cnt %llu ops %llu units %llu build %.1fus plan %.1fus\n",used,c.cnt,(unsigned long long)n,(unsigned long long)nu,
      std::chrono::duration<double,std::micro>(t1-t0).count()/N,std::chrono::duration<double,std::micro>(t2-t1).count()/N);
  }
}
