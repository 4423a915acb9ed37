// TEST INFRASTRUCTURE: the few zbackup types integration/gpu_backup_creator.hh
// names, restated minimally so the adapter compiles and runs in tests (the
// real headers need the generated zbackup.pb.h and libprotobuf).  Same
// names and call signatures as /root/reference/nocopy.hh.
#pragma once
class NoCopy {
 protected:
  NoCopy() {}
 private:
  NoCopy(const NoCopy&);
  NoCopy& operator=(const NoCopy&);
};
