# Compiles the reference's reader (Viterbi_impl/data_reader.cpp + HMM.h) straight from the
# read-only checkout, with a dumper main written here, into oracle/_ref/ (git-ignored).
# Only the reader is buildable: the reference's Viterbi arithmetic needs SuiteSparse:GraphBLAS,
# which is neither installed nor vendored ("Oracle").
REF ?= /root/reference
CXX ?= g++
_ref/ref_reader_dump: ref_reader_dump.cpp $(REF)/Viterbi_impl/data_reader.cpp
	mkdir -p _ref
	$(CXX) -std=c++20 -O2 -I$(REF)/Viterbi_impl -o $@ ref_reader_dump.cpp $(REF)/Viterbi_impl/data_reader.cpp
