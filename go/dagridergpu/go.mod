module github.com/xenowits/dag-rider/dagridergpu

go 1.21
