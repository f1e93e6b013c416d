module gossipgpu

go 1.19
