module gossipref

go 1.20
