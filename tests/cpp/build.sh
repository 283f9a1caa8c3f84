#!/bin/bash
# Build the C++ drop-in test (needs liborbamd.so and the oracle built). Output: tests/cpp/build/test_dropin
set -e
R=$(cd "$(dirname "$0")/../.." && pwd)
mkdir -p "$R/tests/cpp/build"
g++ -std=c++14 -O1 -pthread -Wall -Wno-unused-function \
  -I "$R/tests/cpp/cvmin" -I "$R/tests/cpp/mock" -I "$R/cooperative-orb-slam_amd/host" -I "$R/include" -I "$R/oracle" \
  "$R/tests/cpp/test_dropin.cpp" "$R/cooperative-orb-slam_amd/host/ORBextractor.cc" \
  "$R/cooperative-orb-slam_amd/host/ORBmatcher_amd.cc" "$R/cooperative-orb-slam_amd/host/ORBmatcher_base_amd.cc" \
  "$R/cooperative-orb-slam_amd/host/ORBmatcher_projection_amd.cc" "$R/cooperative-orb-slam_amd/host/Frame_stereo_amd.cc" \
  "$R/cooperative-orb-slam_amd/host/MapPoint_distinctive_amd.cc" "$R/cooperative-orb-slam_amd/host/Frame_bow_amd.cc" \
  "$R/cooperative-orb-slam_amd/host/orbamd_status.cc" \
  -L "$R/cooperative-orb-slam_amd/lib" -lorbamd -L "$R/oracle/build" -lorb_oracle \
  -Wl,-rpath,"$R/cooperative-orb-slam_amd/lib" -Wl,-rpath,"$R/oracle/build" -Wl,-rpath,/opt/rocm/lib \
  -o "$R/tests/cpp/build/test_dropin"
# the drop-ins without a usable device (CPU: must not throw, reference "nothing found" results)
g++ -std=c++14 -O1 -pthread -Wall -Wno-unused-function \
  -I "$R/tests/cpp/cvmin" -I "$R/tests/cpp/mock" -I "$R/cooperative-orb-slam_amd/host" -I "$R/include" \
  "$R/tests/cpp/test_nodevice.cpp" "$R/cooperative-orb-slam_amd/host/ORBextractor.cc" \
  "$R/cooperative-orb-slam_amd/host/ORBmatcher_amd.cc" "$R/cooperative-orb-slam_amd/host/ORBmatcher_base_amd.cc" \
  "$R/cooperative-orb-slam_amd/host/ORBmatcher_projection_amd.cc" "$R/cooperative-orb-slam_amd/host/Frame_stereo_amd.cc" \
  "$R/cooperative-orb-slam_amd/host/MapPoint_distinctive_amd.cc" "$R/cooperative-orb-slam_amd/host/Frame_bow_amd.cc" \
  "$R/cooperative-orb-slam_amd/host/orbamd_status.cc" \
  -L "$R/cooperative-orb-slam_amd/lib" -lorbamd \
  -Wl,-rpath,"$R/cooperative-orb-slam_amd/lib" -Wl,-rpath,/opt/rocm/lib \
  -o "$R/tests/cpp/build/test_nodevice"
# a stock reader of mvImagePyramid: the extractor WITHOUT the drop-in stereo (the device pyramid's reader)
g++ -std=c++14 -O1 -pthread -Wall -Wno-unused-function \
  -I "$R/tests/cpp/cvmin" -I "$R/tests/cpp/mock" -I "$R/cooperative-orb-slam_amd/host" -I "$R/include" -I "$R/oracle" \
  "$R/tests/cpp/test_pyramid_reader.cpp" "$R/cooperative-orb-slam_amd/host/ORBextractor.cc" \
  "$R/cooperative-orb-slam_amd/host/orbamd_status.cc" \
  -L "$R/cooperative-orb-slam_amd/lib" -lorbamd -L "$R/oracle/build" -lorb_oracle \
  -Wl,-rpath,"$R/cooperative-orb-slam_amd/lib" -Wl,-rpath,"$R/oracle/build" -Wl,-rpath,/opt/rocm/lib \
  -o "$R/tests/cpp/build/test_pyramid_reader"
# the slot codec (host only, no GPU needed to run)
g++ -std=c++14 -O1 -Wall -Wno-unused-function \
  -I "$R/tests/cpp/cvmin" -I "$R/tests/cpp/mock" -I "$R/cooperative-orb-slam_amd/host" -I "$R/include" \
  "$R/tests/cpp/test_slot.cpp" "$R/cooperative-orb-slam_amd/host/KeyFrameSlot_amd.cc" \
  -L "$R/cooperative-orb-slam_amd/lib" -lorbamd \
  -Wl,-rpath,"$R/cooperative-orb-slam_amd/lib" -Wl,-rpath,/opt/rocm/lib \
  -o "$R/tests/cpp/build/test_slot"
# per-call latency of the host C ABI vs the oracle, from C++ (tools/run_latency.sh, profiles/)
g++ -std=c++14 -O2 -Wall -I "$R/include" -I "$R/oracle" "$R/tests/cpp/bench_latency.cpp" \
  -L "$R/cooperative-orb-slam_amd/lib" -lorbamd -L "$R/oracle/build" -lorb_oracle \
  -Wl,-rpath,"$R/cooperative-orb-slam_amd/lib" -Wl,-rpath,"$R/oracle/build" -Wl,-rpath,/opt/rocm/lib \
  -o "$R/tests/cpp/build/bench_latency"
# the drop-in class's per-call latency in its default (eager mvImagePyramid) form, and a stereo pair on two threads
g++ -std=c++14 -O2 -pthread -Wall -Wno-unused-function \
  -I "$R/tests/cpp/cvmin" -I "$R/cooperative-orb-slam_amd/host" -I "$R/include" -I "$R/oracle" \
  "$R/tests/cpp/bench_dropin_latency.cpp" "$R/cooperative-orb-slam_amd/host/ORBextractor.cc" \
  "$R/cooperative-orb-slam_amd/host/orbamd_status.cc" \
  -L "$R/cooperative-orb-slam_amd/lib" -lorbamd -L "$R/oracle/build" -lorb_oracle \
  -Wl,-rpath,"$R/cooperative-orb-slam_amd/lib" -Wl,-rpath,"$R/oracle/build" -Wl,-rpath,/opt/rocm/lib \
  -o "$R/tests/cpp/build/bench_dropin_latency"
