bash tools/trace_autofit.sh   # rocprofv3 kernel trace of one autoFit step over 65 536 C2 series
