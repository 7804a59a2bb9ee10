// np_results.h -- output files of a run, in the reference's formats (src/np_results.cpp:39-196,
// include/np_results.h), so that its scripts (scripts/collect.sh, scripts/analyze.m) read them:
//   <workspace><path>/<basename><k>.txt      the items of cluster k, one "x y ... " line each
//   <workspace><path>/<basename>.txt         Octave text: matrix mu (K x D), 3-d matrix sigma
//   <workspace><path>/<basename>.score.txt   purity / Rand index / adjusted Rand index
//   <workspace>LATEST -> <path>              symlink to the latest run
// Clusters are written in ascending id order (the reference iterates an unordered_map).  The
// reference hard-codes 2 columns / "2 2 K" in the Octave header (np_results.cpp:126,156); D is
// written here, which is the same for the reference's 2-d data.
#pragma once

#include <string>
#include <vector>

#include "np_host.h"

class Results {
   public:
    Results(const membertrix &trix, const std::vector<int> &ground_truth);
    void write(const std::string &workspace, const std::string &path, const std::string &basename);
    const clustering_performance &performance() const { return _perf; }

   private:
    void writeOctave(const std::string &fname) const;
    const membertrix &_trix;
    std::vector<int> _gt;
    clustering_performance _perf;
};
